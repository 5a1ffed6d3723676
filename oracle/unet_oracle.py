"""Functional CPU restatement of the reference hot path (TEST INFRASTRUCTURE — see oracle/__init__).

Written from the reference's documented behaviour, as plain aten calls on a flat state_dict:

  depthwise 3^3 conv      unet3d.py:16-17   conv3d(groups=C, padding=1, no bias)
  grouped / dense 3^3     unet3d.py:26-34,43-60  conv3d(groups=G or 1, padding=1, no bias)
  pointwise 1^3 conv      unet3d.py:18      conv3d 1x1x1, no bias
  InstanceNorm3d(affine)  unet3d.py:51,62,72  per-(n,c) biased var, eps=1e-5, no running stats
  LeakyReLU(0.01)         unet3d.py:52,63
  ResidualBlock           unet3d.py:77-93   sc(x); lrelu(IN1(pw1(dw1 x))); [dropout]; IN2(pw2(dw2 .)) + sc; lrelu
  DownBlock               unet3d.py:106-111 maxpool3d(2,2) then RB
  UpBlock                 unet3d.py:126-143 convT(k2,s2,bias); pad-to-skip; cat([up, skip]); RB
  Lightweight3DUNet       unet3d.py:204-223 init, down1..3, bottleneck, up1..3, out_conv(bias), sigmoid
  FocalTverskyLoss        losses.py:30-54   global tp/fp/fn over the whole batch; (1-TI)^gamma

Dropout3d (unet3d.py:66) is channel-wise Bernoulli; the oracle takes an explicit per-(n,c) keep
mask so a caller can reproduce any RNG stream; `None` = eval / p=0.
"""
import torch
import torch.nn.functional as F

EPS = 1e-5
SLOPE = 0.01


def _in(x, w, b):
    return F.instance_norm(x, weight=w, bias=b, eps=EPS)


def conv3(sd, pre, x):
    """ResidualBlock.conv1 / conv2 (unet3d.py:43-60), told apart by the parameter names:
    DepthwiseSeparableConv3d (:12-23: depthwise groups=C then pointwise 1x1), GroupedConv3d
    (:26-34: conv3d groups=G, G = Cin / weight.shape[1]) or a dense nn.Conv3d (:49, :60)."""
    cin = x.shape[1]
    if pre + "depthwise.weight" in sd:
        h = F.conv3d(x, sd[pre + "depthwise.weight"], padding=1, groups=cin)
        return F.conv3d(h, sd[pre + "pointwise.weight"])
    if pre + "conv.weight" in sd:
        w = sd[pre + "conv.weight"]
        return F.conv3d(x, w, padding=1, groups=cin // w.shape[1])
    return F.conv3d(x, sd[pre + "weight"], padding=1)


def residual_block(sd, pre, x, drop_mask=None, drop_p=0.0):
    """unet3d.py:77-93.  `pre` is the state_dict prefix (e.g. 'down1.res_block.')."""
    if pre + "shortcut.0.weight" in sd:
        r = F.conv3d(x, sd[pre + "shortcut.0.weight"])
        r = _in(r, sd[pre + "shortcut.1.weight"], sd[pre + "shortcut.1.bias"])
    else:
        r = x
    h = conv3(sd, pre + "conv1.", x)
    h = F.leaky_relu(_in(h, sd[pre + "norm1.weight"], sd[pre + "norm1.bias"]), SLOPE)
    if drop_mask is not None:
        h = h * drop_mask[:, :, None, None, None] / (1.0 - drop_p)
    h = conv3(sd, pre + "conv2.", h)
    h = _in(h, sd[pre + "norm2.weight"], sd[pre + "norm2.bias"])
    return F.leaky_relu(h + r, SLOPE)


def down_block(sd, pre, x, **kw):
    return residual_block(sd, pre + "res_block.", F.max_pool3d(x, 2, 2), **kw)


def up_block(sd, pre, x, skip, **kw):
    u = F.conv_transpose3d(x, sd[pre + "up.weight"], sd[pre + "up.bias"], stride=2)
    if u.shape != skip.shape:                                   # unet3d.py:130-138
        dd, dh, dw = (skip.shape[i] - u.shape[i] for i in (2, 3, 4))
        u = F.pad(u, [dw // 2, dw - dw // 2, dh // 2, dh - dh // 2, dd // 2, dd - dd // 2])
    return residual_block(sd, pre + "res_block.", torch.cat([u, skip], 1), **kw)


def unet_forward(sd, x, drop_masks=None, drop_p=0.0, return_logits=False):
    """unet3d.py:204-223.  drop_masks: optional dict block-prefix -> [N, C] keep mask."""
    dm = drop_masks or {}

    def kw(name):
        return {"drop_mask": dm.get(name), "drop_p": drop_p}

    x1 = residual_block(sd, "init_conv.", x, **kw("init_conv."))
    x2 = down_block(sd, "down1.", x1, **kw("down1.res_block."))
    x3 = down_block(sd, "down2.", x2, **kw("down2.res_block."))
    x4 = down_block(sd, "down3.", x3, **kw("down3.res_block."))
    h = residual_block(sd, "bottleneck.", x4, **kw("bottleneck."))
    h = up_block(sd, "up1.", h, x3, **kw("up1.res_block."))
    h = up_block(sd, "up2.", h, x2, **kw("up2.res_block."))
    h = up_block(sd, "up3.", h, x1, **kw("up3.res_block."))
    z = F.conv3d(h, sd["out_conv.weight"], sd["out_conv.bias"])
    return z if return_logits else torch.sigmoid(z)


def focal_tversky(pred, target, alpha=0.7, beta=0.3, gamma=0.75, smooth=1e-6):
    """losses.py:30-54: sums over ALL voxels of the batch (pred.view(-1))."""
    assert abs(alpha + beta - 1.0) < 1e-6, f"alpha + beta must equal 1.0, got {alpha + beta}"
    p = pred.reshape(-1)
    t = target.reshape(-1)
    tp = (p * t).sum()
    fp = (p * (1 - t)).sum()
    fn = ((1 - p) * t).sum()
    ti = (tp + smooth) / (tp + alpha * fn + beta * fp + smooth)
    return (1 - ti) ** gamma


def ftl_sums(pred, target):
    """(tp, fp, fn) of losses.py:40-42 as a float64 [3] tensor."""
    p = pred.reshape(-1).double()
    t = target.reshape(-1).double()
    return torch.stack([(p * t).sum(), (p * (1 - t)).sum(), ((1 - p) * t).sum()])


def ftl_grad_closed_form(pred, target, alpha=0.7, beta=0.3, gamma=0.75, smooth=1e-6, sums=None):
    """dL/dp_i in closed form; depends only on t_i and the 3 global sums.
    `sums` overrides the (tp, fp, fn) of `pred` (e.g. the all-reduced sums of a sharded batch)."""
    t = target.reshape(-1).double()
    tp, fp, fn = (sums if sums is not None else ftl_sums(pred, target)).double()
    dn = tp + alpha * fn + beta * fp + smooth
    ti = (tp + smooth) / dn
    dti = (t * dn - (tp + smooth) * (t * (1 - alpha) + beta * (1 - t))) / (dn * dn)
    g = -gamma * (1 - ti) ** (gamma - 1) * dti
    return g.reshape(pred.shape)


def param_names(enc=(16, 32, 64, 128), use_depthwise_separable=True, use_grouped=True, groups=8):
    """Parameter names/shapes in reference registration order (unet3d.py:146-202); the conv
    kinds of each block follow unet3d.py:43-60 (the first block never groups, :163-167)."""
    out = []

    def conv(pre, cin, cout, grouped_ok):
        if use_depthwise_separable:
            out.append((pre + "depthwise.weight", (cin, 1, 3, 3, 3)))
            out.append((pre + "pointwise.weight", (cout, cin, 1, 1, 1)))
        elif grouped_ok:
            out.append((pre + "conv.weight", (cout, cin // groups, 3, 3, 3)))
        else:
            out.append((pre + "weight", (cout, cin, 3, 3, 3)))

    def rb(pre, cin, cout, grouped=True):
        g = use_grouped and grouped and groups > 1
        conv(pre + "conv1.", cin, cout, g and cin >= groups and cout >= groups)
        out.append((pre + "norm1.weight", (cout,)))
        out.append((pre + "norm1.bias", (cout,)))
        conv(pre + "conv2.", cout, cout, g and cout >= groups)
        out.append((pre + "norm2.weight", (cout,)))
        out.append((pre + "norm2.bias", (cout,)))
        if cin != cout:
            out.append((pre + "shortcut.0.weight", (cout, cin, 1, 1, 1)))
            out.append((pre + "shortcut.1.weight", (cout,)))
            out.append((pre + "shortcut.1.bias", (cout,)))

    c0, c1, c2, c3 = enc
    rb("init_conv.", 1, c0, grouped=False)
    rb("down1.res_block.", c0, c1)
    rb("down2.res_block.", c1, c2)
    rb("down3.res_block.", c2, c3)
    rb("bottleneck.", c3, c3)
    for name, ci, co in (("up1.", c3, c2), ("up2.", c2, c1), ("up3.", c1, c0)):
        out.append((name + "up.weight", (ci, ci // 2, 2, 2, 2)))
        out.append((name + "up.bias", (ci // 2,)))
        rb(name + "res_block.", ci, co)
    out.append(("out_conv.weight", (1, c0, 1, 1, 1)))
    out.append(("out_conv.bias", (1,)))
    return out
