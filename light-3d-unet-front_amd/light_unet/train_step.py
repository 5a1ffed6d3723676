"""The reference training hot loop body (trainer.py:222-232: model(images) -> criterion ->
zero_grad -> backward -> optimizer.step) as one engine-level step on the C-ABI kernels.

Unlike the per-parameter autograd path of Lightweight3DUNet.forward (kept for drop-in use by
the reference Trainer), this runs forward, FocalTversky, backward and FlatAdamW directly on the
flat parameter / gradient buffers, with no host synchronisation, so that the whole step can be
captured into hipGraphs (`capture()`), and with the data-parallel exchange placed exactly where
the math needs it:
  * exact mode (default): all-reduce(SUM) of the 3 Focal-Tversky sums after the forward, so
    every rank computes the loss of the GLOBAL batch (losses.py:40-46 semantics); gradients are
    then all-reduced with SUM (the global loss is one function of all ranks' voxels);
  * local mode: each rank's own loss, gradients averaged (plain DDP).
Both collectives are RCCL over xGMI (torch.distributed backend "nccl") on one flat buffer each:
24 B and 0.87 MB (3.25 MB for the 32->256 model) per step.
"""
import os

import torch
import torch.distributed as dist

from . import _native as nat
from .exchange import check_mode, exchange_ftl_sums, exchange_grads, world_size
from .optim import FlatAdamW


def _rccl(group):
    """True when the step's collectives run on RCCL (torch backend "nccl")."""
    return dist.is_available() and dist.is_initialized() and dist.get_backend(group) == "nccl"


class TrainStep:
    def __init__(self, model, loss_cfg=None, lr=1e-4, weight_decay=1e-5, betas=(0.9, 0.999),
                 eps=1e-8, group=None, ftl_mode="exact", distributed=True, dtype=None,
                 force_exchange=False, capture_collectives=None):
        """dtype: activation storage of the step (torch.float32 or torch.bfloat16; default the
        model's compute_dtype, else fp32).  Master weights, AdamW state, gradients and the loss
        stay fp32.
        force_exchange: run the data-parallel step (FocalTversky sums and gradient all-reduces,
        separate update launch) even in a one-rank process group -- the RCCL path on one GPU.
        capture_collectives: capture() records the collectives into the step's one hipGraph
        instead of enqueuing them eagerly between three graph segments.  None (default): capture
        them for the forced one-rank RCCL probe (the only captured-collective form measured on
        hardware: world-1 RCCL, BENCH_r04 `exchange_us`: +12.5 us per step captured, +28.6 us
        segmented), and at world > 1 only with L3U_CAPTURE_COLLECTIVES=1 (no multi-rank
        captured replay has been recorded yet, so the eager segments stay the default there);
        L3U_EAGER_COLLECTIVES=1 forces the segments everywhere.  gloo collectives run on the
        host and always stay eager."""
        loss_cfg = loss_cfg or {}
        self.alpha = float(loss_cfg.get("alpha", 0.7))
        self.beta = float(loss_cfg.get("beta", 0.3))
        self.gamma = float(loss_cfg.get("gamma", 0.75))
        self.smooth = float(loss_cfg.get("smooth", 1e-6))
        assert abs(self.alpha + self.beta - 1.0) < 1e-6
        check_mode(ftl_mode)
        self.model = model
        self.engine = model.engine
        self.act_dtype = dtype or model.compute_dtype or torch.float32
        self.engine.set_act_dtype(self.act_dtype)
        self.flat = model.flat_parameters()
        self.gflat = torch.zeros_like(self.flat)
        # the update launch also advances the Dropout3d counter (no counter launch per step)
        self.opt = FlatAdamW(self.flat, self.gflat, lr=lr, betas=betas, eps=eps,
                             weight_decay=weight_decay, tick_counter=model._rng_counter)
        self.group = group
        # distributed=False: a rank-local step (no exchange) even inside a process group
        self.world = world_size(group) if distributed else 1
        self.force = bool(force_exchange and distributed)
        # the exchange protocol runs (collectives, no fused update) on > 1 rank or when forced
        self.exchange = self.world > 1 or self.force
        if capture_collectives is None:
            capture_collectives = self.exchange and _rccl(group) and \
                os.environ.get("L3U_EAGER_COLLECTIVES", "0") != "1" and \
                (self.world == 1 or os.environ.get("L3U_CAPTURE_COLLECTIVES", "0") == "1")
        self.capture_collectives = bool(capture_collectives)
        self.ftl_mode = ftl_mode
        dev = self.flat.device
        self.loss = torch.zeros((), dtype=torch.float32, device=dev)
        self._graphs = None

    # ----------------------------------------------------------------- pieces
    def _fwd(self, x, t):
        # the out_conv launch also produces the FocalTversky partials (losses.py:40-42)
        N, S = x.shape[0], x[0].numel()
        nparts = N * nat.query("l3u_outconv_nblocks", S)
        part = torch.empty(nparts * 3, dtype=torch.float32, device=x.device)
        self.engine.set_act_dtype(self.act_dtype)
        p, sv = self.engine.forward(self.flat, x, training=self.model.training,
                                    dropout_p=self.model.dropout_p,
                                    counter=self.model._rng_counter, bump_counter=False,
                                    save=True, target=t,
                                    ftl_part=part)
        if not self.exchange:
            # one process: the out_conv backward reduces the partials itself (no reduce launch)
            return p, sv, (part, nparts)
        sums = torch.empty(3, dtype=torch.float64, device=p.device)
        nat.call("l3u_ftl_reduce", part.data_ptr(), nparts, sums.data_ptr(), nat.stream())
        return p, sv, sums

    def _bwd(self, p, sv, t, sums):
        # dL/dp is formed inside the out_conv backward from t and the (global) sums; the same
        # launch writes the loss value (losses.py:52-54)
        abgs = (self.alpha, self.beta, self.gamma, self.smooth)
        if isinstance(sums, tuple):   # (partials, count): reduced inside the out_conv backward
            ftl = (t, None, abgs, self.loss, sums[0], sums[1])
        else:
            ftl = (t, sums, abgs, self.loss)
        # one process: the gradient reduction launch also applies the AdamW update
        self.engine.backward(self.flat, self.gflat, sv, None, need_dx=False, ftl=ftl,
                             opt=None if self.exchange else self.opt)
        return self.engine.applied_update

    def _grad_exchange(self):
        if self.exchange:
            exchange_grads(self.gflat, self.ftl_mode, self.group, force=self.force)

    def _sums_exchange(self, sums):
        if self.exchange:
            exchange_ftl_sums(sums, self.ftl_mode, self.group, force=self.force)

    def _check_flat(self):
        if self.model._flat is not self.flat:
            raise RuntimeError("the model's parameters were re-homed (e.g. .to() to another "
                               "device/dtype) after this TrainStep was built; build a new one")

    # ----------------------------------------------------------------- eager step
    def __call__(self, x, t):
        """One step on device tensors x, t [N,1,D,H,W]; returns the device loss (no sync)."""
        self._check_flat()
        p, sv, sums = self._fwd(x, t)
        self._sums_exchange(sums)
        if not self._bwd(p, sv, t, sums):
            self._grad_exchange()
            self.opt.step()
        return self.loss

    # ----------------------------------------------------------------- hipGraph step
    def capture(self, x_static, t_static, warmup=2):
        """Capture the step into hipGraphs over static input buffers.  With the exchange, the
        collectives stay eager between graph segments: [fwd+sums] -> allreduce(sums) ->
        [loss+bwd] -> allreduce(grads) -> [adamw], unless capture_collectives (RCCL captured in
        the one graph).  Without it (one process) the step is one graph."""
        self.xs, self.ts = x_static, t_static
        # warm-up runs full steps (arena sizing, kernel loading); they must leave no trace: the
        # parameters, the AdamW state and counters and the Dropout3d counter are restored, so
        # capture() is side-effect free even on unfilled static buffers
        self._check_flat()
        state = [self.flat, self.opt.m, self.opt.v, self.opt.step_t, self.opt.ticket,
                 self.model._rng_counter, self.loss]
        saved = [t.clone() for t in state]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self(self.xs, self.ts)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        with torch.no_grad():
            for t, c in zip(state, saved):
                t.copy_(c)
        torch.cuda.synchronize()
        pool = torch.cuda.graph_pool_handle()
        # thread-local capture: with a process group, the RCCL watchdog thread keeps querying
        # its work events while this thread captures, which a global-mode capture turns into
        # "operation not permitted when stream is capturing" in that thread (an abort)
        mode = "thread_local"
        if not self.exchange or self.capture_collectives:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=pool, capture_error_mode=mode):
                self(self.xs, self.ts)
            self._graphs = [g]
        else:
            g1, g2, g3 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, pool=pool, capture_error_mode=mode):
                self._cap_p, self._cap_sv, self._cap_sums = self._fwd(self.xs, self.ts)
            with torch.cuda.graph(g2, pool=pool, capture_error_mode=mode):
                self._bwd(self._cap_p, self._cap_sv, self.ts, self._cap_sums)
            with torch.cuda.graph(g3, pool=pool, capture_error_mode=mode):
                self.opt.step()
            self._graphs = [g1, g2, g3]
        torch.cuda.synchronize()

    def replay(self):
        if self._graphs is None:
            raise RuntimeError("call capture() first")
        self._check_flat()
        if len(self._graphs) == 1:
            self._graphs[0].replay()
        else:
            g1, g2, g3 = self._graphs
            g1.replay()
            self._sums_exchange(self._cap_sums)
            g2.replay()
            self._grad_exchange()
            g3.replay()
        return self.loss
