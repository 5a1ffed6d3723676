"""Per-kernel numerics of the C-ABI library against float64 torch-CPU references of the same ops.

Every kernel is called through the C ABI (light_unet._native -> libl3u_hip.so).  Shapes include
ragged volumes (odd, non-multiple-of-4 sizes), strided batch views (zero-copy concat) and the
48^3 / 24^3 production shapes.  Tolerances: fp32 kernels vs fp64 references, rel 1e-5 .. 1e-4 of
the output scale (each output is a short fp32 dot product / stencil sum).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

SLOPE = 0.01


def nat():
    from light_unet import _native
    return _native


def st():
    return torch.cuda.current_stream().cuda_stream


def close(a, b, rtol=1e-5, what=""):
    a = a.detach().double().cpu()
    b = b.detach().double().cpu()
    scale = max(b.abs().max().item(), 1e-30)
    err = (a - b).abs().max().item() / scale
    assert err <= rtol, f"{what}: max err {err:.3e} (rel to {scale:.3e}) > {rtol}"


def make_rec(N, C, gen, drop=False):
    mean = torch.randn(N, C, generator=gen, dtype=torch.float64) * 0.3
    rstd = 0.5 + torch.rand(N, C, generator=gen, dtype=torch.float64)
    g = 1 + 0.2 * torch.randn(N, C, generator=gen, dtype=torch.float64)
    b = 0.2 * torch.randn(N, C, generator=gen, dtype=torch.float64)
    k = torch.ones(N, C, dtype=torch.float64)
    if drop:
        k = torch.where(torch.rand(N, C, generator=gen) < 0.3, 0.0, 1 / 0.7).double()
    rec = torch.zeros(N, C, 8, dtype=torch.float64)
    rec[..., 0], rec[..., 1] = mean, rstd
    rec[..., 2] = k * g * rstd
    rec[..., 3] = k * b
    rec[..., 4], rec[..., 5], rec[..., 6] = k, g, b
    return rec


def xform_ref(y, rec):
    sc = rec[..., 2][:, :, None, None, None]
    sh = rec[..., 3][:, :, None, None, None]
    mu = rec[..., 0][:, :, None, None, None]
    return F.leaky_relu(sc * (y - mu) + sh, SLOPE)


# ------------------------------------------------------------------------------ depthwise
DW_SHAPES = [(2, 3, 7, 6, 9), (1, 2, 5, 5, 5), (2, 4, 12, 12, 12), (4, 16, 48, 48, 48),
             (2, 8, 6, 6, 6), (1, 2, 24, 24, 24), (1, 1, 64, 64, 64),
             # x-quad path edge cases: H not a multiple of the row strip, odd D, WQ odd
             (2, 3, 7, 10, 8), (1, 2, 9, 52, 20), (2, 2, 33, 4, 4), (1, 3, 3, 8, 12),
             # planes above 64 x 64 (LDS-DMA tiles) and W > 128 (register-staged tiles; the
             # IN-fused backward there takes the two-pass form)
             (1, 1, 5, 80, 80), (1, 2, 4, 6, 136)]


@pytest.mark.parametrize("shape", DW_SHAPES)
@pytest.mark.parametrize("mode", [0, 1])
def test_dw3_fwd(cuda, shape, mode):
    N, C, D, H, W = shape
    gen = torch.Generator().manual_seed(1)
    x = torch.randn(shape, generator=gen, dtype=torch.float64)
    w = torch.randn(C, 1, 3, 3, 3, generator=gen, dtype=torch.float64)
    rec = make_rec(N, C, gen, drop=True) if mode else None
    a = xform_ref(x, rec) if mode else x
    ref = F.conv3d(a, w, padding=1, groups=C)
    # strided input view: embed x in a 2C-channel buffer (upper half) like a concat buffer
    S = D * H * W
    buf = torch.zeros(N, 2 * C, S, device=cuda)
    buf[:, C:] = x.reshape(N, C, S).float().to(cuda)
    y = torch.full((N, C, D, H, W), float("nan"), device=cuda)
    wd = w.float().reshape(C, 27).to(cuda)
    recd = rec.float().to(cuda) if mode else None
    nat().call("l3u_dw3_fwd", buf.data_ptr() + 4 * C * S, 2 * C * S, wd.data_ptr(),
               recd.data_ptr() if mode else None, None, y.data_ptr(), C * S, N, C, D, H, W, st())
    torch.cuda.synchronize()
    close(y, ref, 2e-6, f"dw3_fwd{shape} mode{mode}")


@pytest.mark.parametrize("shape", [(2, 3, 7, 10, 8), (4, 16, 48, 48, 48), (2, 8, 6, 6, 6)])
def test_dw3_fwd_inkernel_finalize(cuda, shape):
    """rec finalized inside the stencil kernel from GEMM partials == l3u_in_finalize + rec path,
    and the record stored for the backward equals the standalone finalize (incl. dropout)."""
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(12)
    y1 = (torch.randn(N, C, S, generator=gen) * 2 + 0.5).to(cuda)
    nsb = 5
    chunks = torch.tensor_split(y1.double().cpu(), nsb, dim=2)
    part = torch.stack([torch.stack([torch.full((N, C), float(ch.shape[2]), dtype=torch.float64),
                                     ch.mean(2), ((ch - ch.mean(2, keepdim=True)) ** 2).sum(2)], -1)
                        for ch in chunks], 2).float().contiguous().to(cuda)
    gamma = (1 + 0.2 * torch.randn(C, generator=gen)).to(cuda)
    beta = (0.2 * torch.randn(C, generator=gen)).to(cuda)
    step = torch.tensor([3], dtype=torch.int32, device=cuda)
    w = torch.randn(C, 27, generator=gen).to(cuda)
    rec_a = torch.empty(N * C * 8, device=cuda)
    nat().call("l3u_in_finalize", part.data_ptr(), nsb, gamma.data_ptr(), beta.data_ptr(), 0.3, 77,
               step.data_ptr(), 5, rec_a.data_ptr(), N, C, st())
    ya = torch.empty(N, C, S, device=cuda)
    nat().call("l3u_dw3_fwd", y1.data_ptr(), C * S, w.data_ptr(), rec_a.data_ptr(), None,
               ya.data_ptr(), C * S, N, C, D, H, W, st())
    rec_b = torch.full((N * C * 8,), float("nan"), device=cuda)
    src = nat().NormSrc(part.data_ptr(), nsb, 5, gamma.data_ptr(), beta.data_ptr(), 0.3, 77,
                        step.data_ptr(), rec_b.data_ptr())
    yb = torch.empty(N, C, S, device=cuda)
    nat().call("l3u_dw3_fwd", y1.data_ptr(), C * S, w.data_ptr(), None, nat().norm_src_ptr(src),
               yb.data_ptr(), C * S, N, C, D, H, W, st())
    torch.cuda.synchronize()
    assert torch.equal(rec_a, rec_b)
    assert torch.equal(ya, yb)


@pytest.mark.parametrize("shape", [(4, 16, 48, 48, 48), (2, 16, 24, 24, 24), (1, 4, 9, 20, 24)])
@pytest.mark.parametrize("finalize", [False, True])
def test_dw3_fwd_rank1_input(cuda, shape, finalize):
    """A rank-1 IN-fused input (negative batch stride: one stored channel z, channel c =
    rec[c][7] * z, include/l3u.h "Rank-1 operands"; the first block's y1 = w1[c] * z1) gives the
    bits of the materialised tensor's forward, with the record given or finalized in-kernel."""
    N, C, D, H, W = shape
    if not nat().query("l3u_dw3_bwd_rank1", N, C, D, H, W):
        pytest.skip("no rank-1 form at this shape")
    S = D * H * W
    gen = torch.Generator().manual_seed(14)
    z = torch.randn(N, 1, S, generator=gen).to(cuda)
    rk = (1 + 0.3 * torch.randn(C, generator=gen)).to(cuda)
    ymat = rk[None, :, None] * z                 # the materialised y1 (same float products)
    w = torch.randn(C, 27, generator=gen).to(cuda)
    rec = make_rec(N, C, gen, drop=True).float()
    rec[..., 7] = rk.cpu()[None, :]
    rec = rec.to(cuda).contiguous()
    ya, yb = torch.empty(N, C, S, device=cuda), torch.empty(N, C, S, device=cuda)
    keep = []
    if finalize:
        # the record from (count, mean, M2) partials of the materialised tensor, rank1 = rk
        nsb = 3
        ch = torch.tensor_split(ymat.double().cpu(), nsb, dim=2)
        part = torch.stack([torch.stack([torch.full((N, C), float(c.shape[2]), dtype=torch.float64),
                                         c.mean(2), ((c - c.mean(2, keepdim=True)) ** 2).sum(2)], -1)
                            for c in ch], 2).float().contiguous().to(cuda)
        g = (1 + 0.1 * torch.randn(C, generator=gen)).to(cuda)
        b = (0.1 * torch.randn(C, generator=gen)).to(cuda)
        step = torch.tensor([2], dtype=torch.int32, device=cuda)
        ra, rb = torch.empty(N * C * 8, device=cuda), torch.empty(N * C * 8, device=cuda)
        sa = nat().NormSrc(part.data_ptr(), nsb, 3, g.data_ptr(), b.data_ptr(), 0.2, 5,
                           step.data_ptr(), ra.data_ptr(), None)
        sb = nat().NormSrc(part.data_ptr(), nsb, 3, g.data_ptr(), b.data_ptr(), 0.2, 5,
                           step.data_ptr(), rb.data_ptr(), rk.data_ptr())
        keep += [sa, sb]
        nat().call("l3u_dw3_fwd", ymat.data_ptr(), C * S, w.data_ptr(), None, nat().norm_src_ptr(sa),
                   ya.data_ptr(), C * S, N, C, D, H, W, st())
        nat().call("l3u_dw3_fwd", z.data_ptr(), -S, w.data_ptr(), None, nat().norm_src_ptr(sb),
                   yb.data_ptr(), C * S, N, C, D, H, W, st())
    else:
        nat().call("l3u_dw3_fwd", ymat.data_ptr(), C * S, w.data_ptr(), rec.data_ptr(), None,
                   ya.data_ptr(), C * S, N, C, D, H, W, st())
        nat().call("l3u_dw3_fwd", z.data_ptr(), -S, w.data_ptr(), rec.data_ptr(), None,
                   yb.data_ptr(), C * S, N, C, D, H, W, st())
    torch.cuda.synchronize()
    assert torch.equal(ya, yb), (ya - yb).abs().max().item()


@pytest.mark.parametrize("shape", DW_SHAPES)
@pytest.mark.parametrize("mode", [0, 1])
def test_dw3_bwd(cuda, shape, mode):
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(2)
    x = torch.randn(shape, generator=gen, dtype=torch.float64)
    w = torch.randn(C, 1, 3, 3, 3, generator=gen, dtype=torch.float64)
    dz = torch.randn(shape, generator=gen, dtype=torch.float64)
    rec = make_rec(N, C, gen, drop=True) if mode else None
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    if mode:
        # reference: pre = IN-affine output (un-dropped), a = k * lrelu(pre)
        k = rec[..., 4][:, :, None, None, None]
        sc = (rec[..., 1] * rec[..., 5])[:, :, None, None, None]
        sh = (rec[..., 6] - rec[..., 5] * rec[..., 1] * rec[..., 0])[:, :, None, None, None]
        pre = (sc * xr + sh).detach().requires_grad_(True)
        a = k * F.leaky_relu(pre, SLOPE)
        out = F.conv3d(a, wr, padding=1, groups=C)
        out.backward(dz)
        dpre_ref = pre.grad
        xhat = (x - rec[..., 0][:, :, None, None, None]) * rec[..., 1][:, :, None, None, None]
        s1_ref = dpre_ref.sum(dim=(2, 3, 4))
        s2_ref = (dpre_ref * xhat).sum(dim=(2, 3, 4))
    else:
        out = F.conv3d(xr, wr, padding=1, groups=C)
        out.backward(dz)
    nch = nat().query("l3u_dw3_nchunk", N, C, D, H, W)
    xd = x.float().to(cuda)
    dzd = dz.float().to(cuda)
    wd = w.float().reshape(C, 27).to(cuda)
    init = torch.randn(shape, generator=gen).to(cuda)
    dx = init.clone()
    dwp = torch.full((C * N * nch * 27,), float("nan"), device=cuda)
    inp = torch.full((C * N * nch * 2,), float("nan"), dtype=torch.float64, device=cuda) if mode else None
    recd = rec.float().to(cuda) if mode else None
    acc = 0 if mode else 1
    nat().call("l3u_dw3_bwd", dzd.data_ptr(), C * S, xd.data_ptr(), C * S, wd.data_ptr(),
               recd.data_ptr() if mode else None, dx.data_ptr(), C * S, acc, dwp.data_ptr(),
               inp.data_ptr() if mode else None, N, C, D, H, W, st())
    torch.cuda.synchronize()
    dwsum = dwp.view(C, N * nch, 27).double().sum(1).view(C, 1, 3, 3, 3)
    close(dwsum, wr.grad, 1e-5, f"dw3_bwd dW {shape} mode{mode}")
    if mode:
        close(dx, dpre_ref, 2e-6, "dpre")
        ip = inp.view(C, N, nch, 2).double().sum(2)
        close(ip[..., 0].t(), s1_ref, 1e-5, "sum dpre")
        close(ip[..., 1].t(), s2_ref, 1e-5, "sum dpre*xhat")
    else:
        close(dx, xr.grad + init.double().cpu(), 2e-6, f"dw3_bwd dX {shape}")


# ------------------------------------------------------------------------------ pointwise GEMM
PW_CASES = [(2, 1, 16, 7 * 6 * 9), (2, 16, 16, 1000), (4, 32, 16, 13824), (3, 16, 32, 216),
            (2, 64, 128, 1728), (2, 128, 64, 216), (1, 128, 128, 216), (2, 32, 512, 216),
            (1, 5, 7, 37)]


@pytest.mark.parametrize("case", PW_CASES)
@pytest.mark.parametrize("layout", [0, 1])
def test_pw_fwd(cuda, case, layout):
    N, K, J, S = case
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(N, K, S, generator=gen, dtype=torch.float64)
    wm = torch.randn(J, K, generator=gen, dtype=torch.float64)   # Wm[j][k]
    bias = torch.randn(J, generator=gen, dtype=torch.float64)
    old = torch.randn(N, J, S, generator=gen, dtype=torch.float64)
    ref = torch.einsum("jk,nks->njs", wm, x) + bias[None, :, None]
    w_store = wm if layout == 0 else wm.t().contiguous()
    xd, wdv, bd = x.float().to(cuda), w_store.float().contiguous().to(cuda), bias.float().to(cuda)
    y = torch.full((N, J, S), float("nan"), device=cuda)
    nsb = nat().query("l3u_pw_stat_nsb", K, J, S)
    part = torch.full((N * J * nsb * 3,), float("nan"), device=cuda)
    nat().call("l3u_pw_fwd", xd.data_ptr(), K * S, wdv.data_ptr(), layout, bd.data_ptr(),
               y.data_ptr(), J * S, 0, part.data_ptr(), N, K, J, S, st())
    torch.cuda.synchronize()
    close(y, ref, 1e-5, f"pw_fwd {case} L{layout}")
    # merged statistics == torch mean / biased var per (n, j)
    p = part.view(N, J, nsb, 3).double().cpu()
    cnt = p[..., 0].sum(-1)
    mean = (p[..., 0] * p[..., 1]).sum(-1) / cnt
    m2 = p[..., 2].sum(-1) + (p[..., 0] * (p[..., 1] - mean[..., None]) ** 2).sum(-1)
    var = m2 / cnt
    assert torch.all(cnt == S)
    close(mean, ref.mean(-1), 1e-5, "stat mean")
    close(var, ref.var(-1, unbiased=False), 1e-4, "stat var")
    # accumulate, no bias, no stats
    y2 = old.float().to(cuda)
    nat().call("l3u_pw_fwd", xd.data_ptr(), K * S, wdv.data_ptr(), layout, None, y2.data_ptr(),
               J * S, 1, None, N, K, J, S, st())
    torch.cuda.synchronize()
    close(y2, ref - bias[None, :, None] + old, 1e-5, "pw_fwd accumulate")


@pytest.mark.parametrize("case", PW_CASES)
def test_pw_bwd_weight(cuda, case):
    N, K, J, S = case
    gen = torch.Generator().manual_seed(4)
    x = torch.randn(N, K, S, generator=gen, dtype=torch.float64)
    dy = torch.randn(N, J, S, generator=gen, dtype=torch.float64)
    ref = torch.einsum("njs,nks->jk", dy, x)
    P = nat().query("l3u_pw_bwd_weight_nparts", N, S)
    part = torch.full((P * J * K,), float("nan"), device=cuda)
    xd, dyd = x.float().to(cuda), dy.float().to(cuda)
    nat().call("l3u_pw_bwd_weight", dyd.data_ptr(), J * S, xd.data_ptr(), K * S, part.data_ptr(),
               N, J, K, S, st())
    torch.cuda.synchronize()
    close(part.view(P, J, K).double().sum(0), ref, 1e-5, f"pw_bwd_weight {case}")


# fused 1x1-conv backward: (N, J, K, S, with_in_prologue, accumulate)
PW_BWD_CASES = [
    (2, 16, 1, 6 * 8 * 10, True, False),       # init block conv1 (K = 1, VALU kernel), ragged chunk
    (1, 16, 1, 48 ** 3, True, False),          # ... at 48^3 (256-voxel chunks)
    (2, 32, 1, 24 ** 3, True, True),           # ... two 16-row halves (config 5), accumulate
    (2, 16, 16, 12 ** 3, False, False),
    (1, 16, 32, 24 ** 3, True, False),         # up3 conv1 shape class, multi-iteration chunks
    (2, 32, 16, 6 * 6 * 8, False, True),       # shortcut: accumulate into d(input)
    (2, 32, 64, 8 ** 3, True, False),          # up2 conv1 (NJ 2, NK 4)
    (3, 20, 40, 4 * 5 * 12, True, True),       # partial tiles in J and K
    (2, 64, 32, 12 ** 3, True, False),         # wide form: down2 conv1
    (2, 64, 128, 12 ** 3, False, True),        # up1 shortcut
    (2, 128, 128, 6 ** 3, True, False),        # bottleneck conv1
    (1, 128, 64, 6 ** 3, False, False),
    (2, 64, 40, 5 * 6 * 8, True, True),        # ragged K, S not a multiple of 64
    # wide form on big volumes (config 5's 32^3 / 16^3 levels): several 64-voxel tiles per
    # workgroup, the last block partial
    (1, 64, 128, 32 ** 3, True, False),
    (2, 128, 64, 16 ** 3, False, True),
    (1, 64, 40, 71 * 64 - 60, True, True),
]


@pytest.mark.parametrize("case", PW_BWD_CASES)
def test_pw_bwd_fused(cuda, case):
    N, J, K, S, pro, acc = case
    assert nat().query("l3u_pw_bwd_supported", J, K, S) == 1
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(N, K, S, generator=gen, dtype=torch.float64)
    w = torch.randn(J, K, generator=gen, dtype=torch.float64) / K ** 0.5
    dpre = torch.randn(N, J, S, generator=gen, dtype=torch.float64)
    if pro:   # dY = InstanceNorm backward of dpre (the in_bwd_apply reference above)
        y = torch.randn(N, J, S, generator=gen, dtype=torch.float64) * 1.5 + 0.2
        g = 1 + 0.3 * torch.randn(J, generator=gen, dtype=torch.float64)
        yr = y.clone().requires_grad_(True)
        F.instance_norm(yr, weight=g, eps=1e-5).backward(dpre)
        dy = yr.grad
        m = y.mean(-1)
        rs = 1 / torch.sqrt(y.var(-1, unbiased=False) + 1e-5)
        rec = torch.zeros(N, J, 8, dtype=torch.float64)
        rec[..., 0], rec[..., 1], rec[..., 5] = m, rs, g.expand(N, J)
        xhat = (y - m[..., None]) * rs[..., None]
        nch = 3
        part_in = torch.zeros(J, N, nch, 2, dtype=torch.float64)
        part_in[:, :, 1, 0] = dpre.sum(-1).t()
        part_in[:, :, 1, 1] = (dpre * xhat).sum(-1).t()
    else:
        dy = dpre
    dx0 = torch.randn(N, K, S, generator=gen, dtype=torch.float64) if acc else torch.zeros(N, K, S,
                                                                                            dtype=torch.float64)
    ref_dx = torch.einsum("jk,njs->nks", w, dy) + dx0
    ref_dw = torch.einsum("njs,nks->jk", dy, x)
    P = nat().query("l3u_pw_bwd_nparts", N, J, K, S)
    part = torch.full((P * J * K,), float("nan"), device=cuda)
    xd, wd, dd = x.float().to(cuda), w.float().to(cuda), dpre.float().to(cuda)
    dx = dx0.float().to(cuda) if acc else torch.full((N, K, S), float("nan"), device=cuda)
    if pro:
        yd, recd, pid = y.float().to(cuda), rec.float().to(cuda), part_in.to(cuda)
        pro_args = (yd.data_ptr(), J * S, recd.data_ptr(), pid.data_ptr(), nch)
    else:
        pro_args = (None, 0, None, None, 0)
    nat().call("l3u_pw_bwd", dd.data_ptr(), J * S, *pro_args, xd.data_ptr(), K * S, wd.data_ptr(),
               dx.data_ptr(), K * S, 1 if acc else 0, part.data_ptr(), N, J, K, S, st())
    torch.cuda.synchronize()
    close(dx, ref_dx, 1e-5, f"pw_bwd dx {case}")
    close(part.view(P, J, K).double().sum(0), ref_dw, 2e-5, f"pw_bwd dw {case}")


@pytest.mark.parametrize("case", [(4, 64, 64, 32, 12 ** 3), (4, 128, 128, 64, 6 ** 3), (2, 64, 128, 64, 12 ** 3),
                                  (2, 128, 40, 24, 5 * 6 * 8)])
def test_pw_bwd2_equals_two_calls(cuda, case):
    """l3u_pw_bwd2 (a block's conv2.pointwise and shortcut backwards in one launch) gives the two
    plain l3u_pw_bwd calls' dX and weight-gradient partials bit for bit."""
    N, J, Ka, Kb, S = case
    assert nat().query("l3u_pw_bwd2_supported", J, S) == 1
    gen = torch.Generator().manual_seed(15)
    r = lambda *s: torch.randn(*s, generator=gen).to(cuda)  # noqa: E731
    dya, xa, wa, dyb, xb, wb = r(N, J, S), r(N, Ka, S), r(J, Ka), r(N, J, S), r(N, Kb, S), r(J, Kb)
    P = nat().query("l3u_pw_bwd_nparts", N, J, Ka, S)
    assert P == nat().query("l3u_pw_bwd_nparts", N, J, Kb, S)
    out = []
    for paired in (True, False):
        dxa, dxb = torch.full((N, Ka, S), float("nan"), device=cuda), torch.full((N, Kb, S), float("nan"), device=cuda)
        pa, pb = torch.full((P * J * Ka,), float("nan"), device=cuda), torch.full((P * J * Kb,), float("nan"), device=cuda)
        if paired:
            nat().call("l3u_pw_bwd2", dya.data_ptr(), J * S, xa.data_ptr(), Ka * S, wa.data_ptr(), dxa.data_ptr(),
                       Ka * S, 0, pa.data_ptr(), Ka, dyb.data_ptr(), J * S, xb.data_ptr(), Kb * S, wb.data_ptr(),
                       dxb.data_ptr(), Kb * S, 0, pb.data_ptr(), Kb, N, J, S, st())
        else:
            for dy, x, w, dx, p, K in ((dya, xa, wa, dxa, pa, Ka), (dyb, xb, wb, dxb, pb, Kb)):
                nat().call("l3u_pw_bwd", dy.data_ptr(), J * S, None, 0, None, None, 0, x.data_ptr(), K * S,
                           w.data_ptr(), dx.data_ptr(), K * S, 0, p.data_ptr(), N, J, K, S, st())
        torch.cuda.synchronize()
        out.append((dxa, dxb, pa, pb))
    for a, b in zip(*out):
        assert torch.equal(a, b)


def test_pw_bwd_matches_unfused(cuda):
    """The fused call reproduces in_bwd_apply + pw_fwd(data) + pw_bwd_weight to fp32 rounding."""
    N, J, K, S = 2, 16, 32, 12 ** 3
    gen = torch.Generator().manual_seed(12)
    x = torch.randn(N, K, S, generator=gen).to(cuda)
    w = torch.randn(J, K, generator=gen).to(cuda)
    dy = torch.randn(N, J, S, generator=gen).to(cuda)
    P = nat().query("l3u_pw_bwd_weight_nparts", N, S)
    p1, p2 = torch.empty(P * J * K, device=cuda), torch.empty(P * J * K, device=cuda)
    dx1, dx2 = torch.empty(N, K, S, device=cuda), torch.empty(N, K, S, device=cuda)
    nat().call("l3u_pw_bwd", dy.data_ptr(), J * S, None, 0, None, None, 0, x.data_ptr(), K * S,
               w.data_ptr(), dx1.data_ptr(), K * S, 0, p1.data_ptr(), N, J, K, S, st())
    nat().call("l3u_pw_fwd", dy.data_ptr(), J * S, w.data_ptr(), 1, None, dx2.data_ptr(), K * S, 0,
               None, N, J, K, S, st())
    nat().call("l3u_pw_bwd_weight", dy.data_ptr(), J * S, x.data_ptr(), K * S, p2.data_ptr(), N, J,
               K, S, st())
    torch.cuda.synchronize()
    close(dx1, dx2, 1e-6, "dx fused vs unfused")
    close(p1.view(P, J, K).sum(0), p2.view(P, J, K).sum(0), 1e-5, "dw fused vs unfused")


# ------------------------------------------------------------------------------ InstanceNorm
def test_in_finalize_and_dropout(cuda):
    N, C, nsb = 3, 5, 7
    gen = torch.Generator().manual_seed(5)
    vals = torch.randn(N, C, nsb, 40, generator=gen, dtype=torch.float64) * 2 + 1
    part = torch.stack([torch.full((N, C, nsb), 40.0, dtype=torch.float64), vals.mean(-1),
                        ((vals - vals.mean(-1, keepdim=True)) ** 2).sum(-1)], -1)
    gamma = torch.randn(C, generator=gen, dtype=torch.float64)
    beta = torch.randn(C, generator=gen, dtype=torch.float64)
    rec = torch.empty(N * C * 8, device=cuda)
    pd = part.float().to(cuda)
    gd, bd = gamma.float().to(cuda), beta.float().to(cuda)
    nat().call("l3u_in_finalize", pd.data_ptr(), nsb, gd.data_ptr(), bd.data_ptr(), 0.0, 1, None, 0,
               rec.data_ptr(), N, C, st())
    torch.cuda.synchronize()
    r = rec.view(N, C, 8).double().cpu()
    flat = vals.reshape(N, C, -1)
    mean, var = flat.mean(-1), flat.var(-1, unbiased=False)
    rstd = 1 / torch.sqrt(var + 1e-5)
    close(r[..., 0], mean, 1e-5, "mean")
    close(r[..., 1], rstd, 1e-5, "rstd")
    close(r[..., 2], gamma * rstd, 1e-5, "scale")
    close(r[..., 3], beta.expand(N, C), 1e-6, "shift")
    # dropout: channel keep mask with scale 1/(1-p), fraction ~ p, deterministic per step
    N2, C2 = 64, 64
    part2 = torch.tensor([1.0, 0.0, 1.0]).repeat(N2 * C2).to(cuda)
    step = torch.tensor([7], dtype=torch.int32, device=cuda)
    recs = []
    for _ in range(2):
        rr = torch.empty(N2 * C2 * 8, device=cuda)
        nat().call("l3u_in_finalize", part2.data_ptr(), 1, None, None, 0.25, 123, step.data_ptr(), 3,
                   rr.data_ptr(), N2, C2, st())
        recs.append(rr.view(N2, C2, 8).cpu())
    k = recs[0][..., 4]
    assert torch.equal(recs[0], recs[1])
    uk = np.unique(k.numpy())
    assert all(np.isclose(v, 0.0) or np.isclose(v, 1 / 0.75, rtol=1e-6) for v in uk), uk
    frac = (k == 0).double().mean().item()
    assert 0.2 < frac < 0.3, frac
    step += 1
    rr = torch.empty(N2 * C2 * 8, device=cuda)
    nat().call("l3u_in_finalize", part2.data_ptr(), 1, None, None, 0.25, 123, step.data_ptr(), 3,
               rr.data_ptr(), N2, C2, st())
    assert not torch.equal(rr.view(N2, C2, 8).cpu()[..., 4], k)


@pytest.mark.parametrize("shortcut", [True, False])
@pytest.mark.parametrize("shape", [(2, 3, 5, 6, 7), (2, 16, 12, 12, 12), (4, 16, 48, 48, 48)])
def test_norm_act_fwd_bwd(cuda, shape, shortcut):
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(6)
    y2 = torch.randn(N, C, S, generator=gen, dtype=torch.float64)
    r = torch.randn(N, C, S, generator=gen, dtype=torch.float64)
    dout = torch.randn(N, C, S, generator=gen, dtype=torch.float64)
    g2 = 1 + 0.3 * torch.randn(C, generator=gen, dtype=torch.float64)
    b2 = 0.3 * torch.randn(C, generator=gen, dtype=torch.float64)
    gr = 1 + 0.3 * torch.randn(C, generator=gen, dtype=torch.float64)
    br = 0.3 * torch.randn(C, generator=gen, dtype=torch.float64)
    y2r, rr = y2.clone().requires_grad_(True), r.clone().requires_grad_(True)
    g2r, b2r, grr, brr = (t.clone().requires_grad_(True) for t in (g2, b2, gr, br))
    res = F.instance_norm(rr, weight=grr, bias=brr, eps=1e-5) if shortcut else rr
    out = F.leaky_relu(F.instance_norm(y2r, weight=g2r, bias=b2r, eps=1e-5) + res, SLOPE)
    out.backward(dout)

    def rec_of(v, g, b):
        m = v.mean(-1)
        rs = 1 / torch.sqrt(v.var(-1, unbiased=False) + 1e-5)
        rc = torch.zeros(N, C, 8, dtype=torch.float64)
        rc[..., 0], rc[..., 1] = m, rs
        rc[..., 2] = g * rs
        rc[..., 3] = b
        rc[..., 4], rc[..., 5], rc[..., 6] = 1, g.expand(N, C), b.expand(N, C)
        return rc.float().to(cuda)

    rec2 = rec_of(y2, g2, b2)
    recr = rec_of(r, gr, br) if shortcut else None
    y2d, rd, dd = y2.float().to(cuda), r.float().to(cuda), dout.float().to(cuda)
    o = torch.empty(N, C, S, device=cuda)
    nat().call("l3u_norm_act_fwd", y2d.data_ptr(), C * S, rec2.data_ptr(), None, rd.data_ptr(),
               C * S, recr.data_ptr() if shortcut else None, None, 1 if shortcut else 0,
               o.data_ptr(), C * S, N, C, S, st())
    # same output when the records are finalized in-kernel from (count, mean, M2) partials
    def src_of(v, g, b, rec_out):
        part = torch.stack([torch.full((N, C), float(S), dtype=torch.float64), v.mean(-1),
                            ((v - v.mean(-1, keepdim=True)) ** 2).sum(-1)], -1).float().to(cuda)
        gd, bd = g.float().to(cuda), b.float().to(cuda)
        return nat().NormSrc(part.data_ptr(), 1, 0, gd.data_ptr(), bd.data_ptr(), 0.0, 0, None,
                             rec_out.data_ptr()), (part, gd, bd)
    ro2 = torch.empty(N * C * 8, device=cuda)
    ror = torch.empty(N * C * 8, device=cuda)
    s2, keep2 = src_of(y2, g2, b2, ro2)
    sr, keepr = src_of(r, gr, br, ror)
    o2 = torch.empty(N, C, S, device=cuda)
    nat().call("l3u_norm_act_fwd", y2d.data_ptr(), C * S, None, nat().norm_src_ptr(s2), rd.data_ptr(),
               C * S, None, nat().norm_src_ptr(sr) if shortcut else None, 1 if shortcut else 0,
               o2.data_ptr(), C * S, N, C, S, st())
    torch.cuda.synchronize()
    close(o2, out, 2e-6, "norm_act out (in-kernel finalize)")
    close(ro2.view(N, C, 8)[..., :4], rec2.view(N, C, 8)[..., :4], 1e-5, "stored rec2")
    nb = nat().query("l3u_norm_act_nblocks", S)
    part = torch.empty(C * N * nb * 3, dtype=torch.float64, device=cuda)
    nat().call("l3u_norm_act_bwd_reduce", dd.data_ptr(), C * S, o.data_ptr(), C * S, y2d.data_ptr(),
               C * S, rec2.data_ptr(), rd.data_ptr(), C * S, recr.data_ptr() if shortcut else None,
               part.data_ptr(), N, C, S, st())
    dy2 = torch.empty(N, C, S, device=cuda)
    dr = torch.empty(N, C, S, device=cuda)
    nat().call("l3u_norm_act_bwd_apply", dd.data_ptr(), C * S, o.data_ptr(), C * S,
               y2d.data_ptr(), C * S, rec2.data_ptr(), rd.data_ptr(), C * S,
               recr.data_ptr() if shortcut else None, part.data_ptr(), dy2.data_ptr(), C * S,
               dr.data_ptr(), C * S, N, C, S, st())
    torch.cuda.synchronize()
    close(o, out, 2e-6, "norm_act out")
    close(dy2, y2r.grad, 1e-4, "dy2")
    close(dr, rr.grad, 1e-4, "dr")
    p = part.view(C, N, nb, 3).double().sum((1, 2)).cpu()
    close(p[:, 0], b2r.grad, 1e-5, "dbeta2")
    close(p[:, 1], g2r.grad, 1e-5, "dgamma2")
    if shortcut:
        close(p[:, 2], grr.grad, 1e-5, "dgamma_r")


@pytest.mark.parametrize("shape,shortcut,with_src", [((2, 3, 4, 6, 8), True, False),
                                                    ((4, 16, 48, 48, 48), False, True),
                                                    ((2, 32, 12, 12, 12), True, True)])
def test_norm_act_pool_fwd(cuda, shape, shortcut, with_src):
    """l3u_norm_act_pool_fwd == l3u_norm_act_fwd followed by l3u_maxpool2_fwd, bit for bit."""
    N, C, D, H, W = shape
    S, So = D * H * W, D * H * W // 8
    gen = torch.Generator().manual_seed(16)
    y2 = torch.randn(N, C, S, generator=gen).to(cuda)
    r = torch.randn(N, C, S, generator=gen).to(cuda)
    if with_src:   # in-kernel finalize from (count, mean, M2) partials
        keep = []

        def src_of(v):
            part = torch.stack([torch.full((N, C), float(S), device=cuda), v.mean(-1),
                                ((v - v.mean(-1, keepdim=True)) ** 2).sum(-1)], -1).contiguous()
            g = (1 + 0.2 * torch.randn(C, generator=gen)).to(cuda)
            b = (0.2 * torch.randn(C, generator=gen)).to(cuda)
            ro = torch.empty(N * C * 8, device=cuda)
            keep.extend([part, g, b, ro])
            return nat().NormSrc(part.data_ptr(), 1, 0, g.data_ptr(), b.data_ptr(), 0.0, 0, None,
                                 ro.data_ptr())
        s2, sr = src_of(y2), src_of(r)
        recs = (None, nat().norm_src_ptr(s2), None, nat().norm_src_ptr(sr) if shortcut else None)
    else:
        rec2 = torch.rand(N * C, 8, generator=gen).to(cuda)
        recr = torch.rand(N * C, 8, generator=gen).to(cuda)
        recs = (rec2.data_ptr(), None, recr.data_ptr() if shortcut else None, None)
    o1, o2 = torch.empty(N, C, S, device=cuda), torch.empty(N, C, S, device=cuda)
    p1, p2 = torch.empty(N, C, So, device=cuda), torch.empty(N, C, So, device=cuda)
    i1 = torch.empty(N, C, So, dtype=torch.uint8, device=cuda)
    i2 = torch.empty(N, C, So, dtype=torch.uint8, device=cuda)
    nat().call("l3u_norm_act_fwd", y2.data_ptr(), C * S, recs[0], recs[1], r.data_ptr(), C * S,
               recs[2], recs[3], int(shortcut), o1.data_ptr(), C * S, N, C, S, st())
    nat().call("l3u_maxpool2_fwd", o1.data_ptr(), C * S, p1.data_ptr(), C * So, i1.data_ptr(), N, C,
               D, H, W, st())
    nat().call("l3u_norm_act_pool_fwd", y2.data_ptr(), C * S, recs[0], recs[1], r.data_ptr(), C * S,
               recs[2], recs[3], int(shortcut), o2.data_ptr(), C * S, p2.data_ptr(), C * So,
               i2.data_ptr(), N, C, D, H, W, st())
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.equal(p1, p2)
    assert torch.equal(i1, i2)


def test_in_bwd_apply(cuda):
    N, C, D, H, W = 2, 4, 6, 5, 7
    S = D * H * W
    gen = torch.Generator().manual_seed(7)
    y = torch.randn(N, C, S, generator=gen, dtype=torch.float64)
    dpre = torch.randn(N, C, S, generator=gen, dtype=torch.float64)
    g = 1 + 0.3 * torch.randn(C, generator=gen, dtype=torch.float64)
    b = 0.3 * torch.randn(C, generator=gen, dtype=torch.float64)
    yr = y.clone().requires_grad_(True)
    out = F.instance_norm(yr, weight=g, bias=b, eps=1e-5)
    out.backward(dpre)
    m = y.mean(-1)
    rs = 1 / torch.sqrt(y.var(-1, unbiased=False) + 1e-5)
    rec = torch.zeros(N, C, 8, dtype=torch.float64)
    rec[..., 0], rec[..., 1], rec[..., 5] = m, rs, g.expand(N, C)
    xhat = (y - m[..., None]) * rs[..., None]
    nch = 3
    part = torch.zeros(C, N, nch, 2, dtype=torch.float64)
    part[:, :, 0, 0] = dpre.sum(-1).t()
    part[:, :, 0, 1] = (dpre * xhat).sum(-1).t()
    dd, yd = dpre.float().to(cuda), y.float().to(cuda)
    recd, pd = rec.float().to(cuda), part.to(cuda)
    nat().call("l3u_in_bwd_apply", dd.data_ptr(), C * S, yd.data_ptr(), C * S, recd.data_ptr(),
               pd.data_ptr(), nch, dd.data_ptr(), C * S, N, C, S, st())
    torch.cuda.synchronize()
    close(dd, yr.grad, 1e-5, "in_bwd_apply")


# ------------------------------------------------------------------------------ pool / convT
@pytest.mark.parametrize("shape,ties,with_add", [
    ((2, 3, 6, 8, 10), False, True),      # scalar kernels (W % 4 != 0)
    ((4, 16, 48, 48, 48), False, True),   # vector kernels
    ((1, 2, 7, 5, 9), False, True),       # odd sizes: dropped border voxels get 0 (+ add)
    ((2, 3, 6, 8, 12), True, True),       # vector, W/4 odd, tied maxima (first in scan order wins)
    ((2, 4, 12, 12, 12), True, False),    # vector, no add
])
def test_maxpool(cuda, shape, ties, with_add):
    N, C, D, H, W = shape
    gen = torch.Generator().manual_seed(8)
    if ties:
        x = torch.randint(0, 3, shape, generator=gen).double()
    else:
        x = torch.randn(shape, generator=gen, dtype=torch.float64)
    xr = x.clone().requires_grad_(True)
    y = F.max_pool3d(xr, 2, 2)
    dy = torch.randn(y.shape, generator=gen, dtype=torch.float64)
    add = (torch.randn(shape, generator=gen, dtype=torch.float64) if with_add
           else torch.zeros(shape, dtype=torch.float64))
    y.backward(dy)
    So = y.shape[2] * y.shape[3] * y.shape[4]
    S = D * H * W
    xd = x.float().to(cuda)
    yd = torch.empty(N, C, So, device=cuda)
    idx = torch.empty(N, C, So, dtype=torch.uint8, device=cuda)
    nat().call("l3u_maxpool2_fwd", xd.data_ptr(), C * S, yd.data_ptr(), C * So, idx.data_ptr(),
               N, C, D, H, W, st())
    dyd, ad = dy.float().to(cuda), add.float().to(cuda)
    dx = torch.empty(N, C, S, device=cuda)
    nat().call("l3u_maxpool2_bwd", dyd.data_ptr(), C * So, idx.data_ptr(),
               ad.data_ptr() if with_add else None, C * S, dx.data_ptr(), C * S, N, C, D, H, W, st())
    torch.cuda.synchronize()
    close(yd.view(y.shape), y, 1e-7, "maxpool fwd")
    close(dx.view(shape), xr.grad + add, 1e-6, "maxpool bwd")


@pytest.mark.parametrize("case", [(2, 16, 7 * 6 * 9), (4, 16, 48 ** 3), (1, 32, 64 ** 3)])
def test_outconv(cuda, case):
    N, C, S = case
    gen = torch.Generator().manual_seed(10)
    h = torch.randn(N, C, S, generator=gen, dtype=torch.float64)
    w = torch.randn(1, C, generator=gen, dtype=torch.float64) * 0.3
    b = torch.randn(1, generator=gen, dtype=torch.float64)
    hr, wr, br = (t.clone().requires_grad_(True) for t in (h, w, b))
    p = torch.sigmoid(torch.einsum("oc,ncs->nos", wr, hr) + br[None, :, None])
    dp = torch.randn(p.shape, generator=gen, dtype=torch.float64)
    p.backward(dp)
    hd, wd, bd = h.float().to(cuda), w.float().to(cuda), b.float().to(cuda)
    pd = torch.empty(N, 1, S, device=cuda)
    nat().call("l3u_outconv_fwd", hd.data_ptr(), C * S, wd.data_ptr(), bd.data_ptr(), pd.data_ptr(),
               None, None, N, C, S, st())
    nb = nat().query("l3u_outconv_nblocks", S)
    part = torch.empty(N * nb * (C + 1), dtype=torch.float64, device=cuda)
    dh = torch.empty(N, C, S, device=cuda)
    dpd = dp.float().to(cuda)
    nat().call("l3u_outconv_bwd", dpd.data_ptr(), pd.data_ptr(), None, None, 0.0, 0.0, 0.0, 0.0,
               None, hd.data_ptr(), C * S, wd.data_ptr(), dh.data_ptr(), C * S, part.data_ptr(), None,
               N, C, S, st())
    torch.cuda.synchronize()
    close(pd, p, 1e-6, "outconv p")
    close(dh, hr.grad, 1e-5, "outconv dh")
    ps = part.view(N * nb, C + 1).double().sum(0).cpu()
    close(ps[:C], wr.grad[0], 1e-5, "outconv dw")
    close(ps[C:], br.grad, 1e-5, "outconv db")


# ------------------------------------------------------------------------------ FTL
@pytest.mark.parametrize("case", ["rand", "empty", "full", "sat", "params"])
def test_ftl_golden(cuda, golden, case):
    z = golden("ftl.npz")
    p = torch.from_numpy(z[f"{case}/pred"]).to(cuda)
    t = torch.from_numpy(z[f"{case}/target"]).to(cuda)
    a, b, g = (float(v) for v in z[f"{case}/abg"])
    n = p.numel()
    nb = nat().query("l3u_ftl_nblocks", n)
    part = torch.empty(nb * 3, device=cuda)
    sums = torch.empty(3, dtype=torch.float64, device=cuda)
    loss = torch.empty((), device=cuda)
    nat().call("l3u_ftl_sums", p.data_ptr(), t.data_ptr(), n, part.data_ptr(), sums.data_ptr(), st())
    nat().call("l3u_ftl_loss", sums.data_ptr(), a, b, g, 1e-6, loss.data_ptr(), st())
    dp = torch.empty_like(p)
    nat().call("l3u_ftl_bwd", p.data_ptr(), t.data_ptr(), n, sums.data_ptr(), a, b, g, 1e-6, None, 0,
               dp.data_ptr(), st())
    torch.cuda.synchronize()
    assert abs(loss.item() - float(z[f"{case}/loss"])) <= 1e-6 * max(1.0, abs(float(z[f"{case}/loss"])))
    close(dp, torch.from_numpy(z[f"{case}/dpred"]), 1e-5, f"ftl dpred {case}")


def test_reduce_segments(cuda):
    src = torch.arange(1000, dtype=torch.float32, device=cuda)
    src64 = torch.arange(500, dtype=torch.float64, device=cuda) * 0.5
    items64 = torch.tensor([[4, 3, 1, 1, 2, 1, 0, 1]], dtype=torch.int64, device=cuda)
    dst64 = torch.zeros(4, device=cuda)
    nat().call("l3u_reduce_segments", src64.data_ptr(), items64.data_ptr(), 1, dst64.data_ptr(), st())
    torch.cuda.synchronize()
    assert dst64[1].item() == 0.5 * (4 + 5 + 6) and dst64[2].item() == 0.5 * (5 + 6 + 7)
    items = torch.tensor([[0, 4, 10, 1, 3, 0, 0, 0],      # dst[0..2] = sum_i src[i*10 + t]
                          [500, 2, 1, 100, 2, 5, 0, 0],   # dst[5..6] = src[500+100t] + src[501+100t]
                          [7, 1, 1, 1, 1, 7, 1, 0]],      # dst[7] += src[7]
                         dtype=torch.int64, device=cuda)
    dst = torch.full((8,), -1.0, device=cuda)
    nat().call("l3u_reduce_segments", src.data_ptr(), items.data_ptr(), 3, dst.data_ptr(), st())
    torch.cuda.synchronize()
    d = dst.cpu()
    assert d[0] == 0 + 10 + 20 + 30 and d[1] == 1 + 11 + 21 + 31 and d[2] == 2 + 12 + 22 + 32
    assert d[5] == 500 + 501 and d[6] == 600 + 601 and d[3] == -1 and d[7] == 6


CONVT_FUSED = [(2, 128, 64, 6, 6, 6), (2, 64, 32, 12, 12, 12), (1, 32, 16, 24, 24, 24),
               (2, 16, 8, 3, 4, 8), (1, 8, 4, 5, 7, 9), (3, 24, 16, 4, 8, 12)]


@pytest.mark.parametrize("case", CONVT_FUSED)
def test_convt_fwd_fused(cuda, case):
    """l3u_convt_fwd: the GEMM with the scatter + bias in its epilogue, into the lower half of a
    concat buffer (upper half untouched), vs torch conv_transpose3d in fp64."""
    N, Ci, Co, D, H, W = case
    Si = D * H * W
    So = 8 * Si
    gen = torch.Generator().manual_seed(11)
    x = torch.randn(N, Ci, D, H, W, generator=gen, dtype=torch.float64)
    w = torch.randn(Ci, Co, 2, 2, 2, generator=gen, dtype=torch.float64)
    b = torch.randn(Co, generator=gen, dtype=torch.float64)
    y = F.conv_transpose3d(x, w, b, stride=2)
    xd, wd, bd = x.float().to(cuda), w.float().to(cuda), b.float().to(cuda)
    cat = torch.full((N, 2 * Co, So), 7.0, device=cuda)
    nat().call("l3u_convt_fwd", xd.data_ptr(), Ci * Si, wd.data_ptr(), bd.data_ptr(), cat.data_ptr(),
               2 * Co * So, N, Ci, Co, D, H, W, st())
    torch.cuda.synchronize()
    close(cat[:, :Co].reshape(y.shape), y, 1e-5, f"convT fused {case}")
    assert torch.all(cat[:, Co:] == 7.0)


@pytest.mark.parametrize("case", [(2, 16, 4096), (3, 16, 1000), (1, 8, 37)])
def test_outconv_ftl_fused(cuda, case):
    """out_conv forward emitting the FocalTversky partials, and its backward forming dL/dp from
    the global sums in-kernel, vs the oracle (losses.py:30-54 autograd) in fp64."""
    from oracle.unet_oracle import focal_tversky
    N, C, S = case
    gen = torch.Generator().manual_seed(12)
    h = torch.randn(N, C, S, generator=gen, dtype=torch.float64)
    w = torch.randn(1, C, generator=gen, dtype=torch.float64) * 0.3
    b = torch.randn(1, generator=gen, dtype=torch.float64)
    t = (torch.rand(N, 1, S, generator=gen) > 0.8).double()
    hr, wr, br = (v.clone().requires_grad_(True) for v in (h, w, b))
    p = torch.sigmoid(torch.einsum("oc,ncs->nos", wr, hr) + br[None, :, None])
    loss = focal_tversky(p, t)
    loss.backward()
    hd, wd, bd, td = h.float().to(cuda), w.float().to(cuda), b.float().to(cuda), t.float().to(cuda)
    nb = nat().query("l3u_outconv_nblocks", S)
    fpart = torch.full((N * nb * 3,), float("nan"), device=cuda)
    pd = torch.empty(N, 1, S, device=cuda)
    nat().call("l3u_outconv_fwd", hd.data_ptr(), C * S, wd.data_ptr(), bd.data_ptr(), pd.data_ptr(),
               td.data_ptr(), fpart.data_ptr(), N, C, S, st())
    sums = torch.empty(3, dtype=torch.float64, device=cuda)
    nat().call("l3u_ftl_reduce", fpart.data_ptr(), N * nb, sums.data_ptr(), st())
    lossd = torch.empty((), device=cuda)
    nat().call("l3u_ftl_loss", sums.data_ptr(), 0.7, 0.3, 0.75, 1e-6, lossd.data_ptr(), st())
    part = torch.empty(N * nb * (C + 1), dtype=torch.float64, device=cuda)
    dh = torch.empty(N, C, S, device=cuda)
    loss2 = torch.full((), float("nan"), device=cuda)
    nat().call("l3u_outconv_bwd", None, pd.data_ptr(), td.data_ptr(), sums.data_ptr(), 0.7, 0.3, 0.75,
               1e-6, None, hd.data_ptr(), C * S, wd.data_ptr(), dh.data_ptr(), C * S, part.data_ptr(),
               loss2.data_ptr(), N, C, S, st())
    torch.cuda.synchronize()
    assert torch.equal(loss2, lossd)   # the loss written by the backward launch
    pr = p.detach()
    ref_sums = torch.stack([(pr * t).sum(), pr.sum(), t.sum()])
    close(sums.cpu(), ref_sums, 1e-5, "ftl sums")
    assert abs(float(lossd) - float(loss.detach())) <= 1e-5 * abs(float(loss.detach())) + 1e-7
    close(dh, hr.grad, 1e-4, "dh via fused FTL gradient")
    ps = part.view(N * nb, C + 1).double().sum(0).cpu()
    close(ps[:C], wr.grad[0], 1e-4, "dw")
    close(ps[C:], br.grad, 1e-4, "db")
    # the folded form: the backward reduces the forward's partials itself, bit-identically
    part3 = torch.empty_like(part)
    dh3 = torch.empty_like(dh)
    loss3 = torch.full((), float("nan"), device=cuda)
    nat().call("l3u_outconv_bwd_ftl", pd.data_ptr(), td.data_ptr(), fpart.data_ptr(), N * nb, 0.7,
               0.3, 0.75, 1e-6, None, hd.data_ptr(), C * S, wd.data_ptr(), dh3.data_ptr(), C * S,
               part3.data_ptr(), loss3.data_ptr(), N, C, S, st())
    torch.cuda.synchronize()
    assert torch.equal(loss3, lossd) and torch.equal(dh3, dh) and torch.equal(part3, part)


# (N, Ci, Co, D, H, W): the network's three up-blocks (low-res volumes) plus ragged ones
CONVT_ONEPASS = [(2, 32, 16, 8, 8, 8), (2, 64, 32, 6, 6, 8), (1, 128, 64, 3, 3, 4),
                 (2, 24, 8, 5, 6, 4), (4, 64, 32, 12, 12, 12), (2, 16, 8, 4, 4, 12),
                 (1, 128, 64, 16, 16, 16),   # config 5's 16^3 -> 32^3: two tiles per workgroup
                 # the one-read tile kernel (Co 16 / 32): the model's 24^3 up3 (two tiles per
                 # workgroup), ragged volumes (a tile past the end), 16 / 32 / 64-channel blocks,
                 # config 5's 32^3 up3 (four tiles per workgroup)
                 (4, 32, 16, 24, 24, 24), (2, 64, 32, 5, 6, 6), (1, 16, 16, 5, 4, 6),
                 (2, 32, 32, 7, 5, 4), (1, 64, 32, 32, 32, 32),
                 # the Co = 64 staged form (>= 4096 pairs): ragged with a single 16-channel
                 # block, and 8 blocks
                 (2, 16, 64, 16, 15, 18), (2, 128, 64, 16, 16, 16)]


@pytest.mark.parametrize("case", CONVT_ONEPASS)
def test_convt_bwd_onepass(cuda, case):
    """l3u_convt_bwd_fused: data, weight and bias gradients of ConvTranspose3d(k2, s2) in one
    launch, dY gathered in place from a concat gradient, vs torch autograd in fp64."""
    N, Ci, Co, D, H, W = case
    Si = D * H * W
    So = 8 * Si
    gen = torch.Generator().manual_seed(14)
    x = torch.randn(N, Ci, D, H, W, generator=gen, dtype=torch.float64)
    w = torch.randn(Ci, Co, 2, 2, 2, generator=gen, dtype=torch.float64)
    b = torch.randn(Co, generator=gen, dtype=torch.float64)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = F.conv_transpose3d(xr, wr, br, stride=2)
    dy = torch.randn(y.shape, generator=gen, dtype=torch.float64)
    y.backward(dy)
    dcat = torch.full((N, 2 * Co, So), 3.0, device=cuda)
    dcat[:, :Co] = dy.reshape(N, Co, So).float().to(cuda)
    xd, wd = x.float().to(cuda), w.float().to(cuda)
    dx = torch.full((N, Ci, Si), float("nan"), device=cuda)
    P = nat().query("l3u_convt_bwd_fused_nparts", N, Ci, Co, D, H, W)
    assert 0 < P <= N * ((Si + 31) // 32)   # one partial per workgroup of >= 32-voxel tiles
    wp = torch.full((P * Ci * Co * 8,), float("nan"), device=cuda)
    bp = torch.full((P * Co,), float("nan"), device=cuda)
    nat().call("l3u_convt_bwd_fused", dcat.data_ptr(), 2 * Co * So, xd.data_ptr(), Ci * Si,
               wd.data_ptr(), dx.data_ptr(), Ci * Si, wp.data_ptr(), bp.data_ptr(), N, Ci, Co, D, H,
               W, st())
    torch.cuda.synchronize()
    close(dx.view(x.shape), xr.grad, 1e-5, f"convT dX {case}")
    close(wp.view(P, Ci, Co * 8).double().sum(0).view(w.shape), wr.grad, 2e-5, "convT dW")
    close(bp.view(P, Co).double().sum(0), br.grad, 1e-5, "convT db")


@pytest.mark.parametrize("case", CONVT_FUSED)
def test_convt_bwd_fused(cuda, case):
    """l3u_convt_bwd: data gradient with dY gathered in place from the lower half of a concat
    gradient buffer, weight and bias partials, vs torch conv_transpose3d autograd in fp64."""
    N, Ci, Co, D, H, W = case
    Si = D * H * W
    So = 8 * Si
    gen = torch.Generator().manual_seed(13)
    x = torch.randn(N, Ci, D, H, W, generator=gen, dtype=torch.float64)
    w = torch.randn(Ci, Co, 2, 2, 2, generator=gen, dtype=torch.float64)
    b = torch.randn(Co, generator=gen, dtype=torch.float64)
    xr, wr, br = (t.clone().requires_grad_(True) for t in (x, w, b))
    y = F.conv_transpose3d(xr, wr, br, stride=2)
    dy = torch.randn(y.shape, generator=gen, dtype=torch.float64)
    y.backward(dy)
    dcat = torch.full((N, 2 * Co, So), 3.0, device=cuda)
    dcat[:, :Co] = dy.reshape(N, Co, So).float().to(cuda)
    xd, wd = x.float().to(cuda), w.float().to(cuda)
    dx = torch.full((N, Ci, Si), float("nan"), device=cuda)
    P = nat().query("l3u_pw_bwd_weight_nparts", N, Si)
    wp = torch.full((P * Ci * Co * 8,), float("nan"), device=cuda)
    bp = torch.full((P * Co,), float("nan"), device=cuda)
    nat().call("l3u_convt_bwd", dcat.data_ptr(), 2 * Co * So, xd.data_ptr(), Ci * Si, wd.data_ptr(),
               dx.data_ptr(), Ci * Si, wp.data_ptr(), bp.data_ptr(), N, Ci, Co, D, H, W, st())
    torch.cuda.synchronize()
    close(dx.view(x.shape), xr.grad, 1e-5, f"convT dX {case}")
    close(wp.view(P, Ci, Co * 8).double().sum(0).view(w.shape), wr.grad, 1e-5, "convT dW")
    close(bp.view(P, Co).double().sum(0), br.grad, 1e-5, "convT db")


@pytest.mark.parametrize("shape", [(4, 128, 216), (4, 64, 1728), (2, 8, 250), (1, 4, 27)])
@pytest.mark.parametrize("shortcut", [False, True])
def test_norm_act_bwd_one_launch_equals_pair(cuda, shape, shortcut):
    """l3u_norm_act_bwd (one workgroup per plane) == l3u_norm_act_bwd_reduce + _apply, bitwise."""
    N, C, S = shape
    assert nat().query("l3u_norm_act_nblocks", S) == 1
    gen = torch.Generator().manual_seed(41)
    t = lambda: torch.randn(N, C, S, generator=gen).to(cuda)  # noqa: E731
    dout, out, y2, r = t(), t(), t(), t()
    rec2 = make_rec(N, C, gen).float().to(cuda)
    recr = make_rec(N, C, gen).float().to(cuda) if shortcut else None
    rp = recr.data_ptr() if shortcut else None

    def run(one):
        part = torch.full((C * N * 3,), float("nan"), dtype=torch.float64, device=cuda)
        dy2 = torch.full((N, C, S), float("nan"), device=cuda)
        dr = torch.full((N, C, S), float("nan"), device=cuda)
        a = (dout.data_ptr(), C * S, out.data_ptr(), C * S, y2.data_ptr(), C * S, rec2.data_ptr(),
             r.data_ptr(), C * S, rp)
        if one:
            nat().call("l3u_norm_act_bwd", *a, part.data_ptr(), dy2.data_ptr(), C * S, dr.data_ptr(),
                       C * S, N, C, S, st())
        else:
            nat().call("l3u_norm_act_bwd_reduce", *a, part.data_ptr(), N, C, S, st())
            nat().call("l3u_norm_act_bwd_apply", *a, part.data_ptr(), dy2.data_ptr(), C * S,
                       dr.data_ptr(), C * S, N, C, S, st())
        torch.cuda.synchronize()
        return part, dy2, dr

    for a, b in zip(run(True), run(False)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dims", [(4, 64, 12, 12, 12), (2, 8, 8, 8, 8), (1, 4, 4, 6, 8)])
@pytest.mark.parametrize("shortcut", [False, True])
def test_norm_act_bwd_up_equals_maxpool_bwd_then_one_launch(cuda, dims, shortcut):
    """l3u_norm_act_bwd_up (dout = dskip + the next level's MaxPool3d backward, formed on load) ==
    l3u_maxpool2_bwd (with dskip as its addend) followed by l3u_norm_act_bwd, bitwise."""
    N, C, D, H, W = dims
    S = D * H * W
    gen = torch.Generator().manual_seed(43)
    t = lambda *s: torch.randn(*s, generator=gen).to(cuda)  # noqa: E731
    x = t(N, C, D, H, W)
    pooled = torch.empty(N, C, S // 8, device=cuda)
    idx = torch.empty(N, C, S // 8, dtype=torch.uint8, device=cuda)
    nat().call("l3u_maxpool2_fwd", x.data_ptr(), C * S, pooled.data_ptr(), C * S // 8, idx.data_ptr(),
               N, C, D, H, W, st())
    dpool, dskip, out, y2, r = t(N, C, S // 8), t(N, C, S), t(N, C, S), t(N, C, S), t(N, C, S)
    rec2 = make_rec(N, C, gen).float().to(cuda)
    recr = make_rec(N, C, gen).float().to(cuda) if shortcut else None
    rp = recr.data_ptr() if shortcut else None

    def run(up):
        part = torch.full((C * N * 3,), float("nan"), dtype=torch.float64, device=cuda)
        dy2 = torch.full((N, C, S), float("nan"), device=cuda)
        dr = torch.full((N, C, S), float("nan"), device=cuda)
        tail = (out.data_ptr(), C * S, y2.data_ptr(), C * S, rec2.data_ptr(), r.data_ptr(), C * S, rp,
                part.data_ptr(), dy2.data_ptr(), C * S, dr.data_ptr(), C * S, N, C)
        if up:
            nat().call("l3u_norm_act_bwd_up", dskip.data_ptr(), C * S, dpool.data_ptr(), C * S // 8,
                       idx.data_ptr(), *tail, D, H, W, st())
        else:
            dlev = torch.full((N, C, S), float("nan"), device=cuda)
            nat().call("l3u_maxpool2_bwd", dpool.data_ptr(), C * S // 8, idx.data_ptr(), dskip.data_ptr(),
                       C * S, dlev.data_ptr(), C * S, N, C, D, H, W, st())
            nat().call("l3u_norm_act_bwd", dlev.data_ptr(), C * S, *tail, S, st())
        torch.cuda.synchronize()
        return part, dy2, dr

    for a, b in zip(run(True), run(False)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(4, 16, 32, 48 ** 3), (4, 32, 16, 24 ** 3), (2, 16, 8, 1000),
                                   (1, 8, 3, 7 * 9 * 12)])
def test_pw_bwd_tail_equals_apply_then_pw_bwd(cuda, shape):
    """l3u_pw_bwd_tail (the block tail's IN/LeakyReLU backward in the pointwise backward's
    prologue) == l3u_norm_act_bwd_apply followed by l3u_pw_bwd, for conv2.pointwise (sel 1,
    K = J) and the Conv1x1 shortcut (sel 2, accumulate), to fp32 rounding (the per-channel
    means are summed in another order)."""
    N, J, K, S = shape
    gen = torch.Generator().manual_seed(43)
    t = lambda C: torch.randn(N, C, S, generator=gen).to(cuda)  # noqa: E731
    dout, out, y2, r = t(J), t(J), t(J), t(J)
    z2, x = t(J), t(K)
    rec2 = make_rec(N, J, gen).float().to(cuda)
    recr = make_rec(N, J, gen).float().to(cuda)
    w2 = torch.randn(J, J, generator=gen).to(cuda)
    wr = torch.randn(J, K, generator=gen).to(cuda)
    nb = nat().query("l3u_norm_act_nblocks", S)
    part = torch.empty(J * N * nb * 3, dtype=torch.float64, device=cuda)
    a = (dout.data_ptr(), J * S, out.data_ptr(), J * S, y2.data_ptr(), J * S, rec2.data_ptr(),
         r.data_ptr(), J * S, recr.data_ptr())
    nat().call("l3u_norm_act_bwd_reduce", *a, part.data_ptr(), N, J, S, st())
    dy2 = torch.empty(N, J, S, device=cuda)
    dr = torch.empty(N, J, S, device=cuda)
    nat().call("l3u_norm_act_bwd_apply", *a, part.data_ptr(), dy2.data_ptr(), J * S, dr.data_ptr(),
               J * S, N, J, S, st())
    init = t(K)
    for sel, yr, rec, dy, xin, w, K_, acc in ((1, y2, rec2, dy2, z2, w2, J, 0),
                                               (2, r, recr, dr, x, wr, K, 1)):
        npw = nat().query("l3u_pw_bwd_nparts", N, J, K_, S)
        outs = []
        for fused in (False, True):
            dx = init[:, :K_].contiguous().clone() if acc else torch.empty(N, K_, S, device=cuda)
            pp = torch.empty(npw * J * K_, device=cuda)
            if fused:
                nat().call("l3u_pw_bwd_tail", dout.data_ptr(), J * S, out.data_ptr(), J * S,
                           yr.data_ptr(), J * S, rec.data_ptr(), part.data_ptr(), nb, sel,
                           xin.data_ptr(), K_ * S, w.data_ptr(), dx.data_ptr(), K_ * S, acc,
                           pp.data_ptr(), N, J, K_, S, st())
            else:
                nat().call("l3u_pw_bwd", dy.data_ptr(), J * S, None, 0, None, None, 0,
                           xin.data_ptr(), K_ * S, w.data_ptr(), dx.data_ptr(), K_ * S, acc,
                           pp.data_ptr(), N, J, K_, S, st())
            torch.cuda.synchronize()
            outs.append((dx, pp.view(npw, J * K_).double().sum(0)))
        close(outs[1][0], outs[0][0], 1e-5, f"dx sel{sel} {shape}")
        close(outs[1][1], outs[0][1], 1e-5, f"dW sel{sel} {shape}")


@pytest.mark.parametrize("shape", [(4, 16, 48, 48, 48), (2, 8, 5, 6, 8), (1, 16, 7, 3, 12)])
def test_front_fwd(cuda, shape):
    """l3u_front_fwd (first block, one input channel): shortcut r = wr*x, z1 = depthwise3(x),
    y1 = w1*z1 and their (count, mean, M2) partials vs fp64 torch."""
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(45)
    x = torch.randn(N, 1, D, H, W, generator=gen, dtype=torch.float64)
    wdw = torch.randn(1, 1, 3, 3, 3, generator=gen, dtype=torch.float64)
    w1 = torch.randn(C, generator=gen, dtype=torch.float64)
    wr = torch.randn(C, generator=gen, dtype=torch.float64)
    z1 = F.conv3d(x, wdw, padding=1).reshape(N, 1, S)
    y1 = w1[None, :, None] * z1
    r = wr[None, :, None] * x.reshape(N, 1, S)
    nb = nat().query("l3u_front_nblocks", S)
    dev = [t.float().to(cuda).contiguous() for t in (x, wdw, w1, wr)]
    z1d = torch.empty(N, 1, S, device=cuda)
    y1d = torch.empty(N, C, S, device=cuda)
    rd = torch.empty(N, C, S, device=cuda)
    s1 = torch.empty(N * C * nb * 3, device=cuda)
    sr = torch.empty(N * C * nb * 3, device=cuda)
    nat().call("l3u_front_fwd", dev[0].data_ptr(), S, dev[1].data_ptr(), dev[2].data_ptr(),
               dev[3].data_ptr(), z1d.data_ptr(), y1d.data_ptr(), rd.data_ptr(), s1.data_ptr(),
               sr.data_ptr(), None, N, C, D, H, W, st())
    torch.cuda.synchronize()
    close(z1d, z1, 1e-6, "z1")
    close(y1d, y1, 1e-6, "y1")
    close(rd, r, 1e-6, "r")
    for part, ref in ((s1, y1), (sr, r)):
        p = part.view(N, C, nb, 3).double().cpu()
        pad = torch.full((N, C, nb * 1024 - S), float("nan"), dtype=torch.float64)
        blocks = torch.cat([ref, pad], 2).view(N, C, nb, 1024)
        valid = ~torch.isnan(blocks)
        cnt = valid.sum(-1).double()
        mean = torch.where(valid, blocks, 0.0).sum(-1) / cnt
        m2 = torch.where(valid, (blocks - mean[..., None]) ** 2, 0.0).sum(-1)
        assert torch.equal(p[..., 0], cnt)
        close(p[..., 1], mean, 1e-5, "block mean")
        close(p[..., 2], m2, 1e-5, "block M2")


# ------------------------------------------------------------------------------ AdamW
def test_adamw_tick_matches_torch(cuda):
    """l3u_adamw_tick (one launch; the last workgroup advances the counters) == torch.optim.AdamW
    (trainer.py:75-79) to fp32 rounding; the extra counter advances once per call, the ticket
    resets."""
    gen = torch.Generator().manual_seed(12)
    n = 217228
    p0 = torch.randn(n, generator=gen)
    ref = p0.clone().to(cuda).requires_grad_(True)
    opt = torch.optim.AdamW([ref], lr=1e-3, weight_decay=1e-2)
    pb = p0.clone().to(cuda)
    mb, vb = torch.zeros(n, device=cuda), torch.zeros(n, device=cuda)
    sb = torch.zeros(1, dtype=torch.int32, device=cuda)
    ticket = torch.zeros(1, dtype=torch.int32, device=cuda)
    ctr = torch.full((1,), 7, dtype=torch.int32, device=cuda)
    lr = torch.tensor([1e-3], device=cuda)
    for _ in range(5):
        g = torch.randn(n, generator=gen).to(cuda)
        ref.grad = g.clone()
        opt.step()
        nat().call("l3u_adamw_tick", pb.data_ptr(), g.data_ptr(), mb.data_ptr(), vb.data_ptr(), n,
                   lr.data_ptr(), 0.9, 0.999, 1e-8, 1e-2, sb.data_ptr(), 1.0, ticket.data_ptr(),
                   ctr.data_ptr(), st())
    torch.cuda.synchronize()
    assert sb.item() == 5 and ctr.item() == 12 and ticket.item() == 0
    close(pb, ref.detach(), 1e-6, "adamw")


@pytest.mark.parametrize("shape", [(4, 32, 16, 48 ** 3), (4, 64, 32, 24 ** 3), (4, 128, 64, 12 ** 3),
                                   (4, 64, 128, 6 ** 3), (2, 8, 16, 1000)])
def test_pw_fwd2_equals_two_pw_fwd(cuda, shape):
    """l3u_pw_fwd2 (a block's shortcut and conv1.pointwise in one launch) == two l3u_pw_fwd
    calls, bitwise (outputs and statistics partials), with strided (concat-view) inputs."""
    N, K, J, S = shape
    gen = torch.Generator().manual_seed(46)
    xa_full = torch.randn(N, 2 * K, S, generator=gen).to(cuda)   # input as the upper half of a concat
    xa = xa_full[:, K:]
    xb = torch.randn(N, K, S, generator=gen).to(cuda)
    wa = torch.randn(J, K, generator=gen).to(cuda)
    wb = torch.randn(J, K, generator=gen).to(cuda)
    nsb = nat().query("l3u_pw_stat_nsb", K, J, S)

    def bufs():
        return (torch.full((N, J, S), float("nan"), device=cuda),
                torch.full((N * J * nsb * 3,), float("nan"), device=cuda))
    (ya, sa), (yb, sb) = bufs(), bufs()
    nat().call("l3u_pw_fwd", xa.data_ptr(), 2 * K * S, wa.data_ptr(), 0, None, ya.data_ptr(), J * S,
               0, sa.data_ptr(), N, K, J, S, st())
    nat().call("l3u_pw_fwd", xb.data_ptr(), K * S, wb.data_ptr(), 0, None, yb.data_ptr(), J * S, 0,
               sb.data_ptr(), N, K, J, S, st())
    (ya2, sa2), (yb2, sb2) = bufs(), bufs()
    nat().call("l3u_pw_fwd2", xa.data_ptr(), 2 * K * S, wa.data_ptr(), ya2.data_ptr(), J * S,
               sa2.data_ptr(), xb.data_ptr(), K * S, wb.data_ptr(), yb2.data_ptr(), J * S,
               sb2.data_ptr(), N, K, J, S, st())
    torch.cuda.synchronize()
    for a, b in ((ya, ya2), (sa, sa2), (yb, yb2), (sb, sb2)):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_box_copy_pad_and_crop(cuda, dt):
    """l3u_box_copy: F.pad of the ConvTranspose3d output to the skip volume (unet3d.py:130-138,
    diff // 2 before each axis) into a channel range of a concat buffer, and the crop back (the
    pad's backward), bit-exact vs torch (a copy)."""
    sfx = "_bf16" if dt == torch.bfloat16 else ""
    N, C, (d, h, w), (D, H, W) = 2, 3, (10, 8, 6), (11, 9, 7)
    src = torch.randn(N, C, d, h, w, device=cuda).to(dt)
    cat = torch.full((N, 2 * C, D, H, W), 7.0, device=cuda).to(dt)
    oz, oy, ox = (D - d) // 2, (H - h) // 2, (W - w) // 2
    nat().call("l3u_box_copy" + sfx, src.data_ptr(), C * d * h * w, d, h, w, cat.data_ptr(),
               2 * C * D * H * W, D, H, W, oz, oy, ox, N, C, st())
    ref = F.pad(src, [ox, W - w - ox, oy, H - h - oy, oz, D - d - oz])
    back = torch.empty_like(src)
    nat().call("l3u_box_copy" + sfx, cat.data_ptr(), 2 * C * D * H * W, D, H, W, back.data_ptr(),
               C * d * h * w, d, h, w, -oz, -oy, -ox, N, C, st())
    torch.cuda.synchronize()
    assert torch.equal(cat[:, :C], ref)
    assert torch.all(cat[:, C:] == 7.0)
    assert torch.equal(back, src)
