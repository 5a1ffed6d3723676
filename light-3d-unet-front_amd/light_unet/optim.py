"""FlatAdamW — torch.optim.AdamW semantics (trainer.py:75-79) as ONE HIP launch over the flat
parameter buffer of Lightweight3DUNet.

State (exp_avg, exp_avg_sq), the step counter and the learning rate live on the device, so the
whole training step (forward, loss, backward, optimizer) can be captured into a single hipGraph
and replayed; `set_lr` writes the device lr (what a CosineAnnealingLR step changes).
Matches torch.optim.AdamW(amsgrad=False, maximize=False):
    p *= 1 - lr*wd;  m = lerp(m, g, 1-b1);  v = b2*v + (1-b2)*g^2
    p -= lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps)
"""
import torch

from . import _native as nat

ADAMW_TICKET_INTS = 32 * 33   # include/l3u.h L3U_ADAMW_TICKET_INTS


class FlatAdamW:
    def __init__(self, flat_params, flat_grads, lr=1e-3, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=1e-2, grad_scale=1.0, tick_counter=None):
        """tick_counter: an int32 device counter (the model's Dropout3d stream counter) that the
        update launch advances together with its own step count (l3u_adamw_tick: one launch)."""
        nat.require_device(flat_params, flat_grads)
        if flat_params.shape != flat_grads.shape or flat_params.dtype != torch.float32:
            raise ValueError("flat params/grads must be matching fp32 buffers")
        self.p, self.g = flat_params, flat_grads
        self.m = torch.zeros_like(flat_params)
        self.v = torch.zeros_like(flat_params)
        self.step_t = torch.zeros(1, dtype=torch.int32, device=flat_params.device)
        self.lr_t = torch.full((1,), float(lr), dtype=torch.float32, device=flat_params.device)
        self.betas = (float(betas[0]), float(betas[1]))
        self.eps = float(eps)
        self.wd = float(weight_decay)
        self.grad_scale = float(grad_scale)
        self.tick_counter = tick_counter
        # [0]: the update's ticket; the rest: the group tickets of the fused reduce + update
        # (include/l3u.h L3U_ADAMW_TICKET_INTS)
        self.ticket = torch.zeros(ADAMW_TICKET_INTS, dtype=torch.int32, device=flat_params.device)

    def set_lr(self, lr):
        self.lr_t.fill_(float(lr))

    def fused_args(self):
        """(g, p, m, v, lr, beta1, beta2, eps, wd, step, grad_scale, ticket, counter2) of
        l3u_reduce_segments_adamw: the update fused into the gradient reduction launch."""
        return (self.g.data_ptr(), self.p.data_ptr(), self.m.data_ptr(), self.v.data_ptr(),
                self.lr_t.data_ptr(), self.betas[0], self.betas[1], self.eps, self.wd,
                self.step_t.data_ptr(), self.grad_scale, self.ticket.data_ptr(),
                self.tick_counter.data_ptr() if self.tick_counter is not None else None)

    def step(self):
        nat.call("l3u_adamw_tick", self.p.data_ptr(), self.g.data_ptr(), self.m.data_ptr(),
                 self.v.data_ptr(), self.p.numel(), self.lr_t.data_ptr(), self.betas[0],
                 self.betas[1], self.eps, self.wd, self.step_t.data_ptr(), self.grad_scale,
                 self.ticket.data_ptr(),
                 self.tick_counter.data_ptr() if self.tick_counter is not None else None,
                 nat.stream())
