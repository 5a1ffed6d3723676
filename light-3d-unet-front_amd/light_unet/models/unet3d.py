"""Lightweight3DUNet — MI355X (gfx950) drop-in for light_unet/models/unet3d.py of the reference.

Same class names, constructor arguments, submodule tree and therefore identical state_dict keys,
shapes and default initialisation as the reference (unet3d.py:12-229), so reference checkpoints
load unchanged (inferencer.py:49) and `Trainer` (trainer.py:57-79) constructs it as before.

What differs is execution: `Lightweight3DUNet.forward` runs the whole network as one autograd
node whose forward and backward are the hand-written HIP kernels of lib/libl3u_hip.so, scheduled
by `light_unet.engine.UNetEngine`.  The nn.Conv3d / nn.InstanceNorm3d / ... submodules below are
parameter containers only (their own forward is never called on this path).  All parameters are
views into ONE flat fp32 buffer (`flat_parameters()`), which is what the kernels, the fused
AdamW and the single-bucket RCCL all-reduce operate on.

use_depthwise_separable=False (GroupedConv3d / dense nn.Conv3d 3^3 convs, unet3d.py:26-34,43-60)
runs on the csrc/gconv.hip kernels.  Not on the MI355X path (raise NotImplementedError): volumes
whose D, H, W are not multiples of 8 (the pad branch of UpBlock, unet3d.py:130-138).
"""
import torch
import torch.nn as nn

from .. import engine as _engine
from .. import _native as nat


class DepthwiseSeparableConv3d(nn.Module):
    """unet3d.py:12-23 — depthwise 3^3 (groups=C) followed by pointwise 1^3, no bias."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, bias=False):
        super().__init__()
        if kernel_size != 3 or stride != 1 or padding != 1 or bias:
            raise NotImplementedError("MI355X path: depthwise 3x3x3, stride 1, padding 1, no bias")
        self.depthwise = nn.Conv3d(in_channels, in_channels, kernel_size=kernel_size,
                                   stride=stride, padding=padding, groups=in_channels, bias=bias)
        self.pointwise = nn.Conv3d(in_channels, out_channels, kernel_size=1, bias=bias)

    def forward(self, x):
        raise RuntimeError("submodules are parameter containers; call Lightweight3DUNet")


class GroupedConv3d(nn.Module):
    """unet3d.py:26-34 — grouped 3^3 conv (stride 1, padding 1, no bias); runs in the
    csrc/gconv.hip kernels (l3u_gconv3_*)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, padding=1, groups=8,
                 bias=False):
        super().__init__()
        if kernel_size != 3 or stride != 1 or padding != 1 or bias:
            raise NotImplementedError("MI355X path: grouped 3x3x3, stride 1, padding 1, no bias")
        self.conv = nn.Conv3d(in_channels, out_channels, kernel_size=kernel_size,
                              stride=stride, padding=padding, groups=groups, bias=bias)

    def forward(self, x):
        raise RuntimeError("submodules are parameter containers; call Lightweight3DUNet")


class ResidualBlock(nn.Module):
    """unet3d.py:37-93 — same submodule names (conv1, norm1, relu1, conv2, norm2, relu2, dropout,
    shortcut) so parameter names match.  conv1 / conv2 are chosen exactly as the reference does
    (:43-60): depthwise-separable, GroupedConv3d, or a dense nn.Conv3d."""

    def __init__(self, in_channels, out_channels, use_depthwise_separable=True,
                 use_grouped=True, groups=8, dropout_p=0.1):
        super().__init__()
        if use_depthwise_separable:
            self.conv1 = DepthwiseSeparableConv3d(in_channels, out_channels, kernel_size=3, padding=1)
        elif use_grouped and groups > 1 and in_channels >= groups and out_channels >= groups:
            self.conv1 = GroupedConv3d(in_channels, out_channels, kernel_size=3, padding=1, groups=groups)
        else:
            self.conv1 = nn.Conv3d(in_channels, out_channels, kernel_size=3, padding=1, bias=False)
        self.norm1 = nn.InstanceNorm3d(out_channels, affine=True)
        self.relu1 = nn.LeakyReLU(0.01, inplace=True)
        if use_depthwise_separable:
            self.conv2 = DepthwiseSeparableConv3d(out_channels, out_channels, kernel_size=3, padding=1)
        elif use_grouped and groups > 1 and out_channels >= groups:
            self.conv2 = GroupedConv3d(out_channels, out_channels, kernel_size=3, padding=1, groups=groups)
        else:
            self.conv2 = nn.Conv3d(out_channels, out_channels, kernel_size=3, padding=1, bias=False)
        self.norm2 = nn.InstanceNorm3d(out_channels, affine=True)
        self.relu2 = nn.LeakyReLU(0.01, inplace=True)
        self.dropout = nn.Dropout3d(dropout_p) if dropout_p > 0 else None
        if in_channels != out_channels:
            self.shortcut = nn.Sequential(
                nn.Conv3d(in_channels, out_channels, kernel_size=1, bias=False),
                nn.InstanceNorm3d(out_channels, affine=True))
        else:
            self.shortcut = nn.Identity()

    def forward(self, x):
        raise RuntimeError("submodules are parameter containers; call Lightweight3DUNet")


class DownBlock(nn.Module):
    """unet3d.py:96-111"""

    def __init__(self, in_channels, out_channels, use_depthwise_separable=True,
                 use_grouped=True, groups=8, dropout_p=0.1):
        super().__init__()
        self.pool = nn.MaxPool3d(kernel_size=2, stride=2)
        self.res_block = ResidualBlock(in_channels, out_channels,
                                       use_depthwise_separable=use_depthwise_separable,
                                       use_grouped=use_grouped, groups=groups, dropout_p=dropout_p)

    def forward(self, x):
        raise RuntimeError("submodules are parameter containers; call Lightweight3DUNet")


class UpBlock(nn.Module):
    """unet3d.py:114-143"""

    def __init__(self, in_channels, out_channels, use_depthwise_separable=True,
                 use_grouped=True, groups=8, dropout_p=0.1):
        super().__init__()
        self.up = nn.ConvTranspose3d(in_channels, in_channels // 2, kernel_size=2, stride=2)
        self.res_block = ResidualBlock(in_channels, out_channels,
                                       use_depthwise_separable=use_depthwise_separable,
                                       use_grouped=use_grouped, groups=groups, dropout_p=dropout_p)

    def forward(self, x, skip):
        raise RuntimeError("submodules are parameter containers; call Lightweight3DUNet")


class _UNetFunction(torch.autograd.Function):
    """Whole-network autograd node: forward and backward are C-ABI kernel schedules."""

    @staticmethod
    def forward(ctx, model, x, *params):
        flat = model._flat
        model.engine.set_act_dtype(model.act_dtype())
        p, sv = model.engine.forward(flat, x, training=model.training, dropout_p=model.dropout_p,
                                     counter=model._rng_counter, save=True)
        ctx.model = model
        ctx.sv = sv
        return p

    @staticmethod
    def backward(ctx, dp):
        model = ctx.model
        flat = model._flat
        g = torch.empty_like(flat)
        dx = model.engine.backward(flat, g, ctx.sv, dp.contiguous(), need_dx=ctx.needs_input_grad[1])
        ctx.sv = None
        grads = [g[off:off + n].view(shape) for (off, n, shape) in model._slices]
        return (None, dx, *grads)


class Lightweight3DUNet(nn.Module):
    """unet3d.py:146-229 — lightweight 3D U-Net (16 -> 32 -> 64 -> 128) for lesion segmentation."""

    def __init__(self, in_channels=1, out_channels=1, start_channels=16,
                 encoder_channels=[16, 32, 64, 128],
                 use_depthwise_separable=True, use_grouped=True, groups=8,
                 dropout_p=0.1, *, compute_dtype=None):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.encoder_channels = encoder_channels
        self.dropout_p = float(dropout_p) if dropout_p > 0 else 0.0
        kw = dict(use_depthwise_separable=use_depthwise_separable, use_grouped=use_grouped,
                  groups=groups, dropout_p=dropout_p)
        self.init_conv = ResidualBlock(in_channels, encoder_channels[0],
                                       use_depthwise_separable=use_depthwise_separable,
                                       use_grouped=False, groups=groups, dropout_p=dropout_p)
        self.down1 = DownBlock(encoder_channels[0], encoder_channels[1], **kw)
        self.down2 = DownBlock(encoder_channels[1], encoder_channels[2], **kw)
        self.down3 = DownBlock(encoder_channels[2], encoder_channels[3], **kw)
        self.bottleneck = ResidualBlock(encoder_channels[3], encoder_channels[3], **kw)
        self.up1 = UpBlock(encoder_channels[3], encoder_channels[2], **kw)
        self.up2 = UpBlock(encoder_channels[2], encoder_channels[1], **kw)
        self.up3 = UpBlock(encoder_channels[1], encoder_channels[0], **kw)
        self.out_conv = nn.Conv3d(encoder_channels[0], out_channels, kernel_size=1)
        self.sigmoid = nn.Sigmoid()

        self.engine = _engine.UNetEngine(encoder_channels, in_channels, out_channels,
                                         use_depthwise_separable=use_depthwise_separable,
                                         use_grouped=use_grouped, groups=groups)
        # None: fp32, or bf16 under torch.autocast; torch.bfloat16 forces the bf16 path
        self.compute_dtype = None
        if compute_dtype is not None:
            self.engine.set_act_dtype(compute_dtype)
            self.compute_dtype = compute_dtype
        names = [n for n, _ in self.named_parameters()]
        if names != [n for n, _ in self.engine.layout]:
            raise AssertionError("parameter registration order diverged from the engine layout")
        self._slices = [self.engine.offsets[n] for n in names]
        self._flatten()

    # -------------------------------------------------------------- flat parameter storage
    def _flatten(self):
        """Re-home every parameter as a view of one contiguous buffer (after init or .to()).
        When the existing buffer already has the parameters' device and dtype (a no-op .to(),
        or a parameter replaced in place), it is refilled in place and keeps its identity and
        the Dropout3d counter, so a TrainStep / FlatAdamW built on it stays attached."""
        params = list(self.parameters())
        dev = params[0].device
        dt = params[0].dtype
        old = getattr(self, "_flat", None)
        reuse = old is not None and old.device == dev and old.dtype == dt
        flat = old if reuse else torch.empty(self.engine.numel, device=dev, dtype=dt)
        with torch.no_grad():
            for p, (off, n, shape) in zip(params, self._slices):
                dst = flat[off:off + n]
                if p.data_ptr() != dst.data_ptr():
                    dst.copy_(p.detach().reshape(-1))
                p.data = dst.view(shape)
        self._flat = flat
        cnt = getattr(self, "_rng_counter", None)
        if cnt is None or cnt.device != dev:
            self._rng_counter = torch.zeros(1, dtype=torch.int32, device=dev)

    def _is_flat(self):
        base = self._flat.data_ptr()
        for p, (off, n, shape) in zip(self.parameters(), self._slices):
            if p.data_ptr() != base + off * p.element_size() or p.device != self._flat.device:
                return False
        return True

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        self._flatten()
        return out

    def flat_parameters(self):
        """The single fp32 buffer every parameter is a view of (kernel + optimizer + RCCL view)."""
        if not self._is_flat():
            self._flatten()
        return self._flat

    def param_slices(self):
        return dict(zip([n for n, _ in self.named_parameters()], self._slices))

    # -------------------------------------------------------------- forward
    def forward(self, x):
        flat = self.flat_parameters()
        if not x.is_cuda or flat.device != x.device:
            raise nat.NativeError(
                f"Lightweight3DUNet (MI355X path) needs input and model on the same ROCm device; "
                f"got input on {x.device}, model on {flat.device}.  There is no CPU fallback.")
        if flat.dtype != torch.float32:
            raise NotImplementedError("the MI355X path keeps fp32 parameters (bf16 activations: "
                                      "compute_dtype=torch.bfloat16 or torch.autocast)")
        x = x.float()
        if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in self.parameters())):
            return _UNetFunction.apply(self, x, *self.parameters())
        self.engine.set_act_dtype(self.act_dtype())
        p, _ = self.engine.forward(flat, x, training=self.training, dropout_p=self.dropout_p,
                                   counter=self._rng_counter, save=False)
        return p

    def act_dtype(self):
        """Storage dtype of the activations for this call: `compute_dtype` when set, else bf16
        inside torch.autocast("cuda", dtype=torch.bfloat16), else fp32.  Parameters, InstanceNorm
        statistics, the returned probabilities and all accumulation stay fp32 (BASELINE config 3:
        bf16 activations with fp32 master weights)."""
        if self.compute_dtype is not None:
            return self.compute_dtype
        if torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16:
            return torch.bfloat16
        return torch.float32

    def count_parameters(self):
        """Count total and trainable parameters (unet3d.py:225-229)"""
        total = sum(p.numel() for p in self.parameters())
        trainable = sum(p.numel() for p in self.parameters() if p.requires_grad)
        return {"total": total, "trainable": trainable}
