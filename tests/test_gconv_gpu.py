"""Grouped / dense 3^3 conv kernels (csrc/gconv.hip, the use_depthwise_separable=False path of
ResidualBlock, unet3d.py:26-34,43-60) against float64 torch-CPU conv3d of the same op, called
through the C ABI; and the variant networks against the reference's goldens and the oracle.

Tolerances: each output is a <= 27*Cin/G-term fp32 dot product: rel 2e-6 .. 1e-5 of the output
scale; weight gradients sum N*S terms: rel 1e-5; whole-network as tests/test_model_gpu.py.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import unet_oracle as U

pytestmark = pytest.mark.gpu

SLOPE = 0.01


def nat():
    from light_unet import _native
    return _native


def st():
    return torch.cuda.current_stream().cuda_stream


def close(a, b, rtol, what):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = max(b.abs().max().item(), 1e-30)
    err = (a - b).abs().max().item() / scale
    assert err <= rtol, f"{what}: max err {err:.3e} (rel to {scale:.3e}) > {rtol}"


def make_rec(N, C, gen):
    mean = torch.randn(N, C, generator=gen, dtype=torch.float64) * 0.3
    rstd = 0.5 + torch.rand(N, C, generator=gen, dtype=torch.float64)
    g = 1 + 0.2 * torch.randn(N, C, generator=gen, dtype=torch.float64)
    b = 0.2 * torch.randn(N, C, generator=gen, dtype=torch.float64)
    k = torch.where(torch.rand(N, C, generator=gen) < 0.3, 0.0, 1 / 0.7).double()
    rec = torch.zeros(N, C, 8, dtype=torch.float64)
    rec[..., 0], rec[..., 1] = mean, rstd
    rec[..., 2] = k * g * rstd
    rec[..., 3] = k * b
    rec[..., 4], rec[..., 5], rec[..., 6] = k, g, b
    return rec


def pre_act(y, rec):
    """pre = IN-affine output (un-dropped) and a = k * lrelu(pre) (unet3d.py:84-88)"""
    e = lambda i: rec[..., i][:, :, None, None, None]  # noqa: E731
    pre = e(1) * e(5) * (y - e(0)) + e(6)
    return pre, e(4)


# (N, Cin, Cout, G, D, H, W): grouped shapes of the shipped channel plan, dense (G = 1) ones of
# the first block / use_grouped=False, ragged volumes and partial voxel blocks
SHAPES = [(2, 16, 16, 8, 7, 6, 9), (1, 1, 16, 1, 12, 10, 8), (2, 32, 16, 8, 24, 24, 24),
          (4, 128, 128, 8, 6, 6, 6), (1, 16, 16, 1, 8, 8, 8), (2, 8, 16, 4, 5, 5, 5),
          (1, 16, 40, 1, 6, 6, 6), (1, 64, 64, 8, 12, 12, 12),
          # W % 4 == 0 with more than 16 input channels per group: gconv3q_kernel's multi-stage
          # weight path (a barrier + stage_w inside the k loop, the next channel's rows fetched
          # across the stage boundary), LDS-staged (8^3) and global-row (24^3) forms
          (1, 32, 32, 1, 8, 8, 8), (2, 64, 32, 2, 24, 24, 24)]


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("xf", [False, True])
def test_gconv3_fwd(cuda, shape, xf):
    N, Cin, Cout, G, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(N, Cin, D, H, W, generator=gen, dtype=torch.float64)
    w = torch.randn(Cout, Cin // G, 3, 3, 3, generator=gen, dtype=torch.float64) * 0.3
    rec = make_rec(N, Cin, gen) if xf else None
    if xf:
        pre, k = pre_act(x, rec)
        a = k * F.leaky_relu(pre, SLOPE)
    else:
        a = x
    ref = F.conv3d(a, w, padding=1, groups=G)
    nb = nat().query("l3u_gconv3_nblocks", S)
    y = torch.full((N, Cout, S), float("nan"), device=cuda)
    sp = torch.full((N * Cout * nb * 3,), float("nan"), device=cuda)
    recd = rec.float().to(cuda) if xf else None
    xd, wd = x.float().to(cuda), w.float().to(cuda)   # keep the device copies alive
    nat().call("l3u_gconv3_fwd", xd.data_ptr(), Cin * S, wd.data_ptr(),
               recd.data_ptr() if xf else None, y.data_ptr(), Cout * S, sp.data_ptr(), N, Cin, Cout,
               G, D, H, W, st())
    torch.cuda.synchronize()
    close(y.view_as(ref), ref, 1e-5, f"gconv fwd {shape} xf={xf}")
    # (count, mean, M2) partials per 256-voxel block, the l3u_pw_fwd format
    r = ref.reshape(N, Cout, S)
    pad = torch.full((N, Cout, nb * 256 - S), float("nan"), dtype=torch.float64)
    blocks = torch.cat([r, pad], 2).view(N, Cout, nb, 256)
    valid = ~torch.isnan(blocks)
    cnt = valid.sum(-1).double()
    mean = torch.where(valid, blocks, 0.0).sum(-1) / cnt
    m2 = torch.where(valid, (blocks - mean[..., None]) ** 2, 0.0).sum(-1)
    p = sp.view(N, Cout, nb, 3).double().cpu()
    assert torch.equal(p[..., 0], cnt)
    close(p[..., 1], mean, 1e-5, "block mean")
    close(p[..., 2], m2, 1e-5, "block M2")


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_gconv3_bwd(cuda, shape, mode):
    """mode 0: dx = conv^T(dy); 2: dx += conv^T(dy); 1: the IN-fused form (dpre + IN sums).
    The weight gradient is checked in every mode (against the IN-transformed input in mode 1)."""
    N, Cin, Cout, G, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(12)
    x = torch.randn(N, Cin, D, H, W, generator=gen, dtype=torch.float64)
    w = torch.randn(Cout, Cin // G, 3, 3, 3, generator=gen, dtype=torch.float64) * 0.3
    dy = torch.randn(N, Cout, D, H, W, generator=gen, dtype=torch.float64)
    rec = make_rec(N, Cin, gen) if mode == 1 else None
    wr = w.clone().requires_grad_(True)
    if mode == 1:
        pre, k = pre_act(x, rec)
        pre = pre.detach().requires_grad_(True)
        a = k * F.leaky_relu(pre, SLOPE)
        F.conv3d(a, wr, padding=1, groups=G).backward(dy)
        dpre_ref = pre.grad
        xhat = (x - rec[..., 0][:, :, None, None, None]) * rec[..., 1][:, :, None, None, None]
        s1_ref = dpre_ref.sum(dim=(2, 3, 4))
        s2_ref = (dpre_ref * xhat).sum(dim=(2, 3, 4))
    else:
        xr = x.clone().requires_grad_(True)
        F.conv3d(xr, wr, padding=1, groups=G).backward(dy)
    nb = nat().query("l3u_gconv3_nblocks", S)
    P = nat().query("l3u_gconv3_wgrad_nparts", N, S)
    xd, wd, dyd = x.float().to(cuda), w.float().to(cuda), dy.float().to(cuda)
    recd = rec.float().to(cuda) if mode == 1 else None
    init = torch.randn(N, Cin, S, generator=gen).to(cuda)
    dx = init.clone()
    inp = torch.full((Cin * N * nb * 2,), float("nan"), dtype=torch.float64, device=cuda)
    nat().call("l3u_gconv3_bwd_data", dyd.data_ptr(), Cout * S, wd.data_ptr(),
               recd.data_ptr() if mode == 1 else None, xd.data_ptr() if mode == 1 else None, Cin * S,
               dx.data_ptr(), Cin * S, 1 if mode == 2 else 0, inp.data_ptr() if mode == 1 else None,
               N, Cin, Cout, G, D, H, W, st())
    part = torch.full((P * Cout * (Cin // G) * 27,), float("nan"), device=cuda)
    nat().call("l3u_gconv3_bwd_weight", dyd.data_ptr(), Cout * S, xd.data_ptr(), Cin * S,
               recd.data_ptr() if mode == 1 else None, part.data_ptr(), N, Cin, Cout, G, D, H, W, st())
    torch.cuda.synchronize()
    gw = part.view(P, -1).double().sum(0).cpu().view_as(w)
    close(gw, wr.grad, 1e-5, f"gconv dW {shape} mode{mode}")
    if mode == 1:
        close(dx.view_as(dpre_ref), dpre_ref, 2e-6, "dpre")
        ip = inp.view(Cin, N, nb, 2).double().sum(2).cpu()
        close(ip[..., 0].t(), s1_ref, 1e-5, "sum dpre")
        close(ip[..., 1].t(), s2_ref, 1e-5, "sum dpre*xhat")
    else:
        ref = xr.grad + (init.double().cpu().view_as(xr) if mode == 2 else 0)
        close(dx.view_as(ref), ref, 2e-6, f"gconv dX {shape} mode{mode}")


def test_gconv3_rejects_bad_groups(cuda):
    x = torch.zeros(1, 12, 8, device=cuda)
    with pytest.raises(nat().NativeError):
        nat().call("l3u_gconv3_fwd", x.data_ptr(), 12 * 8, x.data_ptr(), None, x.data_ptr(), 12 * 8,
                   None, 1, 12, 12, 8, 2, 2, 2, st())


# ------------------------------------------------------------------------------ whole network
VARIANTS = {"model_g_b2_16.npz": dict(use_depthwise_separable=False, use_grouped=True, groups=8),
            "model_d_b1_16.npz": dict(use_depthwise_separable=False, use_grouped=False, groups=8)}


def _grad_errs(grads, ref):
    errs, num, den = {}, 0.0, 0.0
    for k, g in grads.items():
        gr = ref[k].astype(np.float64)
        d = np.linalg.norm(g.astype(np.float64) - gr)
        errs[k] = d / max(np.linalg.norm(gr), 1e-30)
        num += d * d
        den += float(np.sum(gr * gr))
    return errs, (num / den) ** 0.5


def _oracle_grads(sd, x, t, dtype):
    params = {k: v.clone().to(dtype).requires_grad_(True) for k, v in sd.items()}
    out = U.unet_forward(params, x.to(dtype))
    loss = U.focal_tversky(out, t.to(dtype))
    loss.backward()
    return out.detach(), loss.item(), {k: p.grad.numpy() for k, p in params.items()}


def _run(model, x, t, cuda):
    from light_unet.models.losses import FocalTverskyLoss
    model.train()
    out = model(x.to(cuda))
    loss = FocalTverskyLoss()(out, t.to(cuda))
    model.zero_grad(set_to_none=True)
    loss.backward()
    torch.cuda.synchronize()
    return out.detach().cpu(), loss.item(), {k: p.grad.detach().cpu().numpy()
                                             for k, p in model.named_parameters()}


@pytest.mark.parametrize("fname", sorted(VARIANTS))
def test_variant_model_matches_reference_golden(cuda, golden, fname):
    from light_unet.models.unet3d import Lightweight3DUNet
    z = golden(fname)
    enc = [int(c) for c in z["enc"]]
    m = Lightweight3DUNet(encoder_channels=enc, dropout_p=0.0, **VARIANTS[fname])
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    m.load_state_dict(sd)
    m = m.to(cuda)
    x, t = torch.from_numpy(z["x"]), torch.from_numpy(z["target"])
    o, loss, grads = _run(m, x, t, cuda)
    assert np.abs(o.numpy() - z["out"]).max() <= 1e-3
    assert abs(loss - float(z["loss"])) <= 1e-4 * abs(float(z["loss"]))
    gold = {k: z["g/" + k] for k in grads}
    errs, gerr = _grad_errs(grads, gold)
    _, _, g32 = _oracle_grads(sd, x, t, torch.float32)
    e32, ge32 = _grad_errs(g32, gold)
    assert gerr <= max(1e-3, 2 * ge32), (gerr, ge32)
    bad = {k: (errs[k], e32[k]) for k in errs if errs[k] > max(1e-2, 3 * e32[k])}
    assert not bad, f"gradient errors above tolerance: {bad}"


def test_grouped_model_full_channels_matches_oracle(cuda):
    """The shipped channel plan (16->32->64->128, groups 8; 391,521 parameters) at bs 2, 32^3
    against the fp64 oracle (pinned to the reference by the goldens above)."""
    from light_unet.models.unet3d import Lightweight3DUNet
    torch.manual_seed(42)
    m = Lightweight3DUNet(dropout_p=0.0, use_depthwise_separable=False)
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.to(cuda)
    rng = np.random.default_rng(47)
    x = torch.from_numpy(rng.random((2, 1, 32, 32, 32), dtype=np.float32))
    t = torch.from_numpy((rng.random((2, 1, 32, 32, 32)) > 0.97).astype(np.float32))
    o, loss, grads = _run(m, x, t, cuda)
    ro, rl, rg = _oracle_grads(sd, x, t, torch.float64)
    assert (o.double() - ro).abs().max().item() <= 1e-3
    assert abs(loss - rl) <= 1e-4 * abs(rl)
    errs, gerr = _grad_errs(grads, rg)
    _, _, g32 = _oracle_grads(sd, x, t, torch.float32)
    _, ge32 = _grad_errs(g32, rg)
    assert gerr <= max(1e-3, 2 * ge32), (gerr, ge32)


def test_grouped_trainstep_graph_matches_eager(cuda):
    """TrainStep (graph-captured step, fused AdamW) runs the grouped network; replay is bitwise
    identical to the eager steps, and the loss decreases on a fixed batch."""
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    torch.manual_seed(42)
    sd = Lightweight3DUNet(dropout_p=0.1, use_depthwise_separable=False).state_dict()

    def fresh():
        mm = Lightweight3DUNet(dropout_p=0.1, use_depthwise_separable=False)
        mm.load_state_dict(sd)
        return mm.to(cuda).train()

    rng = np.random.default_rng(48)
    x = torch.from_numpy(rng.random((2, 1, 32, 32, 32), dtype=np.float32)).to(cuda)
    t = torch.from_numpy((rng.random((2, 1, 32, 32, 32)) > 0.97).astype(np.float32)).to(cuda)
    mb = fresh()
    tb = TrainStep(mb, lr=1e-3, weight_decay=1e-5)
    lb = [tb(x, t).item() for _ in range(5)]
    mc = fresh()
    tc = TrainStep(mc, lr=1e-3, weight_decay=1e-5)
    xs, tsb = x.clone(), t.clone()
    tc.capture(xs, tsb, warmup=2)   # side-effect free: the replays start at step 1
    lc = [tc.replay().item() for _ in range(5)]
    assert np.all(np.isfinite(lb))
    np.testing.assert_array_equal(lb, lc)
    assert torch.equal(mb.flat_parameters(), mc.flat_parameters())
