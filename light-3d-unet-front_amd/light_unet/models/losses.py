"""Loss functions — MI355X drop-in for light_unet/models/losses.py of the reference.

`FocalTverskyLoss` (losses.py:11-54) is the hot-path loss: its forward is two HIP launches
(block partials of {sum p*t, sum p, sum t} and a fixed-order fp64 merge, then (1 - TI)^gamma on
the device) and its backward is the closed-form gradient in one elementwise HIP
launch — no host synchronisation anywhere, so it captures into a hipGraph.  Exactly like the
reference, the sums run over ALL voxels of the batch (pred.view(-1)), non-contiguous inputs raise
(as .view(-1) does), alpha + beta must equal 1 (AssertionError, losses.py:28) and an unknown
loss name raises ValueError (losses.py:147).

`CombinedLoss` / `DiceLoss` (losses.py:57-113) are not enabled by any shipped config and are OUT
of the hot-path scope; they are provided for API completeness as compositions of the
FTL kernel and plain device tensor ops.
"""
import torch
import torch.nn as nn

from .. import _native as nat


def _ftl_sums(pred, target):
    n = pred.numel()
    nb = nat.query("l3u_ftl_nblocks", n)
    part = torch.empty(nb * 3, dtype=torch.float32, device=pred.device)
    sums = torch.empty(3, dtype=torch.float64, device=pred.device)
    nat.call("l3u_ftl_sums", pred.data_ptr(), target.data_ptr(), n, part.data_ptr(),
             sums.data_ptr(), nat.stream())
    return sums


class _FTLFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pred, target, alpha, beta, gamma, smooth, reduce_hook, grad_scale=1.0):
        sums = _ftl_sums(pred, target)
        if reduce_hook is not None:            # data-parallel: all-reduce the 3 global sums
            reduce_hook(sums)
        loss = torch.empty((), dtype=torch.float32, device=pred.device)
        nat.call("l3u_ftl_loss", sums.data_ptr(), alpha, beta, gamma, smooth, loss.data_ptr(),
                 nat.stream())
        ctx.save_for_backward(pred, target, sums)
        ctx.abgs = (alpha, beta, gamma, smooth)
        ctx.grad_scale = grad_scale
        return loss

    @staticmethod
    def backward(ctx, gout):
        pred, target, sums = ctx.saved_tensors
        a, b, g, s = ctx.abgs
        gout = gout.contiguous().float()
        if ctx.grad_scale != 1.0:
            gout = gout * ctx.grad_scale
        dp = torch.empty_like(pred)
        nat.call("l3u_ftl_bwd", pred.data_ptr(), target.data_ptr(), pred.numel(), sums.data_ptr(),
                 a, b, g, s, gout.data_ptr(), 0, dp.data_ptr(), nat.stream())
        return dp, None, None, None, None, None, None, None


def _check_inputs(pred, target):
    if not pred.is_contiguous() or not target.is_contiguous():
        # the reference's pred.view(-1) raises on non-contiguous input (losses.py:40-41)
        raise RuntimeError("view size is not compatible with input tensor's size and stride; "
                           "FocalTverskyLoss needs contiguous pred/target (as the reference)")
    if pred.numel() != target.numel():
        raise RuntimeError(f"pred has {pred.numel()} elements but target has {target.numel()}")
    nat.require_device(pred, target)
    if pred.dtype != torch.float32:
        raise NotImplementedError("the MI355X FocalTversky kernel takes fp32 predictions")


class FocalTverskyLoss(nn.Module):
    """
    Focal Tversky Loss for imbalanced segmentation (losses.py:11-54)

    Args:
        alpha: Weight for false negatives (higher = prioritize recall)
        beta: Weight for false positives (higher = prioritize precision)
        gamma: Focal parameter (higher = focus on hard examples)
        smooth: Smoothing factor to avoid division by zero
    """

    def __init__(self, alpha=0.7, beta=0.3, gamma=0.75, smooth=1e-6):
        super().__init__()
        self.alpha = alpha
        self.beta = beta
        self.gamma = gamma
        self.smooth = smooth
        # data-parallel hook: callable(sums_fp64[3]) that all-reduces the sums in place, so every
        # rank forms the loss of the GLOBAL batch (losses.py:40-46 sums over every voxel).  Each
        # rank's backward is then its share of the global loss's gradient: the parameter
        # gradients must be SUMMED over ranks (exchange.exchange_grads(..., "exact")).  Under a
        # reduction that AVERAGES them (torch DDP), set hook_grad_scale = world size.
        self.reduce_hook = None
        self.hook_grad_scale = 1.0
        assert abs(alpha + beta - 1.0) < 1e-6, f"alpha + beta must equal 1.0, got {alpha + beta}"

    def forward(self, pred, target):
        _check_inputs(pred, target)
        target = target.float() if target.dtype != torch.float32 else target
        return _FTLFunction.apply(pred, target, float(self.alpha), float(self.beta),
                                  float(self.gamma), float(self.smooth), self.reduce_hook,
                                  float(self.hook_grad_scale) if self.reduce_hook else 1.0)


class CombinedLoss(nn.Module):
    """losses.py:57-87: w_ftl * FocalTversky + w_bce * BCE over the flattened batch.  Out of the
    hot-path scope (no shipped config enables it); composed from the FTL kernel and torch's BCE."""

    def __init__(self, ftl_weight=0.8, bce_weight=0.2, alpha=0.7, beta=0.3, gamma=0.75):
        super().__init__()
        if abs(ftl_weight + bce_weight - 1.0) >= 1e-6:
            raise AssertionError(f"Weights must sum to 1.0, got {ftl_weight + bce_weight}")
        self.ftl_weight, self.bce_weight = ftl_weight, bce_weight
        self.focal_tversky = FocalTverskyLoss(alpha=alpha, beta=beta, gamma=gamma)
        self.bce = nn.BCELoss()

    def forward(self, pred, target):
        terms = (self.focal_tversky(pred, target), self.bce(pred.view(-1), target.view(-1)))
        return self.ftl_weight * terms[0] + self.bce_weight * terms[1]


class DiceLoss(nn.Module):
    """losses.py:90-113: 1 - (2 sum(p t) + s) / (sum p + sum t + s) over the flattened batch.
    Out of the hot-path scope; plain device tensor ops."""

    def __init__(self, smooth=1e-6):
        super().__init__()
        self.smooth = smooth

    def forward(self, pred, target):
        p, t = pred.view(-1), target.view(-1)
        num = 2.0 * torch.dot(p, t) + self.smooth
        return 1.0 - num / (p.sum() + t.sum() + self.smooth)


_LOSSES = {
    "FocalTverskyLoss": lambda c: FocalTverskyLoss(alpha=c.get("alpha", 0.7), beta=c.get("beta", 0.3),
                                                   gamma=c.get("gamma", 0.75)),
    "DiceLoss": lambda c: DiceLoss(),
}


def get_loss_function(config):
    """losses.py:116-147: build the loss named by config["loss"] (a combined FTL + BCE loss when
    use_combined_loss is set); ValueError for an unknown name."""
    if config.get("use_combined_loss", False):
        w = config.get("combined_loss_weights", {"focal_tversky": 0.8, "bce": 0.2})
        return CombinedLoss(ftl_weight=w["focal_tversky"], bce_weight=w["bce"],
                            alpha=config.get("alpha", 0.7), beta=config.get("beta", 0.3),
                            gamma=config.get("gamma", 0.75))
    name = config.get("name", "FocalTverskyLoss")
    if name not in _LOSSES:
        raise ValueError(f"Unknown loss function: {name}")
    return _LOSSES[name](config)
