"""bf16-storage restatement of the network (TEST INFRASTRUCTURE — see oracle/__init__): the
reference forward / FocalTversky of unet_oracle.py (unet3d.py:12-223, losses.py:30-54), with the
activations rounded to bf16 exactly where the MI355X engine stores them in bf16 (BASELINE
config 3: bf16 activation storage, fp32 arithmetic, fp32 gradients), so that the HIP bf16 network
can be held to a tight bound instead of the fp32 reference's loose one.

Storage points (light_unet/engine.py with the `_bf16` kernels):
  * every stored activation is R(v) = v rounded to bf16 (round to nearest even); consumers read
    the stored value: z1 / z2 (depthwise outputs), y1 / y2 / r (pointwise and shortcut outputs),
    the block output, the pooled input of the next level (MaxPool3d over the stored values), the
    ConvTranspose3d output (the lower half of the concat buffer);
  * InstanceNorm statistics are those of the stored values (pointwise epilogues round first),
    EXCEPT in the first block (l3u_front_fwd, one input channel): y1 = w1 * dw(x) and r = wr * x
    are formed from the fp32 input and the unrounded z1, and their statistics from those unrounded
    values; the backward reads the bf16 copies of x and z1;
  * the normalisation and LeakyReLU / Dropout3d are applied on load (never stored), the network
    input and the out_conv / sigmoid output / loss stay fp32;
  * the backward is fp32 on the stored values: R is the identity for gradients (straight-through),
    the InstanceNorm backward uses x_hat of the stored tensor with the record's mean / rstd.
Computed in float64 (the engine in fp32); the rounding decisions agree except for values within
fp32 rounding of a bf16 tie.
"""
import torch
import torch.nn.functional as F

from .unet_oracle import EPS, SLOPE


class _Round(torch.autograd.Function):
    @staticmethod
    def forward(ctx, v):
        return v.to(torch.bfloat16).to(v.dtype)

    @staticmethod
    def backward(ctx, g):
        return g


def R(v):
    """Stored value: rounded to bf16 in the forward, identity in the backward."""
    return _Round.apply(v)


class Storage:
    """The storage points of one forward.  forced=None: each stored tensor is R(v).  forced = a
    dict of the engine's own stored tensors (key -> tensor): the forward value at each storage
    point is the engine's (teacher forcing, straight-through to v in the backward), and every
    point records (R(v), engine value) so a test can check each op of the chain on the engine's
    own inputs."""

    def __init__(self, forced=None):
        self.forced = forced
        self.pairs = {}

    def __call__(self, v, key):
        if self.forced is None or key not in self.forced:
            return R(v)
        e = self.forced[key].to(v.dtype).reshape(v.shape)
        self.pairs[key] = (R(v).detach(), e)
        return v + (e - v).detach()


class _InRec(torch.autograd.Function):
    """InstanceNorm3d(affine) applied to the stored tensor ys with the record (mean, rstd) of a
    statistics source; backward of the engine (l3u_in_bwd_apply): with xhat = (ys - mean) * rstd,
    dys = gamma * rstd * (g - mean(g) - xhat * mean(g * xhat)), dgamma = sum g * xhat,
    dbeta = sum g."""

    @staticmethod
    def forward(ctx, ys, mean, rstd, gamma, beta):
        xhat = (ys - mean) * rstd
        ctx.save_for_backward(xhat, rstd, gamma)
        return xhat * gamma[None, :, None, None, None] + beta[None, :, None, None, None]

    @staticmethod
    def backward(ctx, g):
        xhat, rstd, gamma = ctx.saved_tensors
        dims = (2, 3, 4)
        gg = g * gamma[None, :, None, None, None]
        m1 = gg.mean(dim=dims, keepdim=True)
        m2 = (gg * xhat).mean(dim=dims, keepdim=True)
        dys = rstd * (gg - m1 - xhat * m2)
        return dys, None, None, (g * xhat).sum(dim=(0,) + dims), g.sum(dim=(0,) + dims)


def _stats(v):
    mean = v.mean(dim=(2, 3, 4), keepdim=True)
    var = v.var(dim=(2, 3, 4), unbiased=False, keepdim=True)
    return mean.detach(), (1.0 / torch.sqrt(var + EPS)).detach()


def in_stored(ys, gamma, beta, src=None):
    """IN of the stored tensor ys with the statistics of `src` (default: ys itself).  With
    src = ys this is exactly autograd's instance_norm of ys (the statistics' gradient included:
    the engine's backward formula is the full one), detached statistics plus the custom backward."""
    mean, rstd = _stats(ys if src is None else src)
    return _InRec.apply(ys, mean, rstd, gamma, beta)


def _weight_only(f, w, x_fwd, x_saved):
    """f(x_fwd, w) in the forward, with the weight gradient of f(x_saved, w) (the kernel's
    backward reads the stored copy x_saved) and the input gradient through x_saved."""
    return f(x_saved, w) + (f(x_fwd, w) - f(x_saved, w)).detach()


def residual_block(sd, pre, x, drop_mask=None, drop_p=0.0, front=False, x_raw=None, st=None):
    """unet3d.py:77-93 with bf16 storage.  front=True: the first block (x_raw the fp32 input, x its
    stored bf16 copy), l3u_front_fwd's semantics.  st: the Storage (storage keys pre + z1, y1, r,
    z2, y2, out)."""
    st = st or Storage()
    cin = x.shape[1]
    dw1, pw1 = sd[pre + "conv1.depthwise.weight"], sd[pre + "conv1.pointwise.weight"]
    if front:
        dwf = lambda v, w: F.conv3d(v, w, padding=1, groups=cin)  # noqa: E731
        z1u = _weight_only(dwf, dw1, x_raw, x)          # dw of the fp32 input
        z1 = st(z1u, pre + "z1")
        y1u = _weight_only(F.conv3d, pw1, z1u, z1)      # w1 * unrounded z1
        y1 = st(y1u, pre + "y1")
        ru = _weight_only(F.conv3d, sd[pre + "shortcut.0.weight"], x_raw, x)
        r = in_stored(st(ru, pre + "r"), sd[pre + "shortcut.1.weight"], sd[pre + "shortcut.1.bias"], src=ru)
        h = in_stored(y1, sd[pre + "norm1.weight"], sd[pre + "norm1.bias"], src=y1u)
    else:
        if pre + "shortcut.0.weight" in sd:
            rs = st(F.conv3d(x, sd[pre + "shortcut.0.weight"]), pre + "r")
            r = in_stored(rs, sd[pre + "shortcut.1.weight"], sd[pre + "shortcut.1.bias"])
        else:
            r = x
        z1 = st(F.conv3d(x, dw1, padding=1, groups=cin), pre + "z1")
        y1 = st(F.conv3d(z1, pw1), pre + "y1")
        h = in_stored(y1, sd[pre + "norm1.weight"], sd[pre + "norm1.bias"])
    h = F.leaky_relu(h, SLOPE)
    if drop_mask is not None:
        h = h * drop_mask[:, :, None, None, None] / (1.0 - drop_p)
    cout = h.shape[1]
    z2 = st(F.conv3d(h, sd[pre + "conv2.depthwise.weight"], padding=1, groups=cout), pre + "z2")
    y2 = st(F.conv3d(z2, sd[pre + "conv2.pointwise.weight"]), pre + "y2")
    h = in_stored(y2, sd[pre + "norm2.weight"], sd[pre + "norm2.bias"])
    return st(F.leaky_relu(h + r, SLOPE), pre + "out")


def unet_forward(sd, x, drop_masks=None, drop_p=0.0, st=None):
    """unet3d.py:204-223 with bf16 activation storage; x fp32 (or fp64) [N, 1, D, H, W] with
    W % 4 == 0 (the shapes l3u_front_fwd takes).  st: a Storage (default: plain rounding);
    storage keys <block prefix> + z1 / y1 / r / z2 / y2 / out and <up prefix> + "u" (the
    ConvTranspose3d output)."""
    assert x.shape[1] == 1 and x.shape[-1] % 4 == 0
    st = st or Storage()
    dm = drop_masks or {}

    def kw(name):
        return {"drop_mask": dm.get(name), "drop_p": drop_p, "st": st}

    x1 = residual_block(sd, "init_conv.", R(x), front=True, x_raw=x, **kw("init_conv."))
    x2 = residual_block(sd, "down1.res_block.", F.max_pool3d(x1, 2, 2), **kw("down1.res_block."))
    x3 = residual_block(sd, "down2.res_block.", F.max_pool3d(x2, 2, 2), **kw("down2.res_block."))
    x4 = residual_block(sd, "down3.res_block.", F.max_pool3d(x3, 2, 2), **kw("down3.res_block."))
    h = residual_block(sd, "bottleneck.", x4, **kw("bottleneck."))
    for up, skip in (("up1.", x3), ("up2.", x2), ("up3.", x1)):
        u = st(F.conv_transpose3d(h, sd[up + "up.weight"], sd[up + "up.bias"], stride=2), up + "u")
        assert u.shape == skip.shape, "the pad branch is not restated here"
        h = residual_block(sd, up + "res_block.", torch.cat([u, skip], 1), **kw(up + "res_block."))
    return torch.sigmoid(F.conv3d(h, sd["out_conv.weight"], sd["out_conv.bias"]))
