"""bf16 activation storage (BASELINE config 3; SURVEY §8b "each has fp32 and bf16 variants").

1. Op twins.  Every _bf16 entry point is run beside its fp32 twin on the SAME inputs: the saved
   activations are drawn, rounded to bf16, and handed to the fp32 call as fp32 and to the bf16
   call as bf16; gradients, weights, records and partial sums are the same fp32 tensors in both
   (the bf16 network stores forward activations in bf16 and keeps every gradient in fp32).  Both
   compute in fp32, so
     * bf16 activation outputs (forward) equal the fp32 outputs rounded to nearest even, to <= 1
       bf16 ulp everywhere (rounding ties, fp32 summation-order differences inside the kernels),
       and exactly on >= 99% of the elements;
     * fp32 outputs (gradients, weight / statistics partials) agree to 1e-5 of the tensor scale,
       1e-2 where the bf16 kernel takes its statistics from the rounded stored values (the IN
       partials of l3u_pw_fwd: the record then normalises exactly what the consumer reads).
2. The network.  The bf16 model (compute_dtype / torch.autocast) against the reference's fp64
   goldens and the fp32 HIP path.  Bounds (SURVEY §8c, bf16 "compare to fp32 with looser bounds,
   reported rather than asserted bit-exact"): output |dp| <= 2e-2 (measured max 9.3e-3, mean
   1.2e-3); loss within 1e-2 relative; the whole parameter gradient within 0.2 relative L2 of the
   fp64 golden and at cosine >= 0.98 to it (measured 0.121-0.133 and 0.991: the bf16-rounded
   pre-activations move ~0.3% of the voxels across the LeakyReLU kink, where the derivative jumps
   100x — with fp32 gradient buffers the error is the same, 0.1327 vs 0.1330 with bf16 ones, so
   it comes from the stored forward activations, not from the gradient storage); thresholded masks identical on every voxel farther than 2e-2 (the output bound)
   from the threshold, and >= 99.5% agreement overall.  The survey's example of >= 99.9% overall
   agreement is not attainable with 8 significant bits per stored activation on these goldens:
   the random-init network's outputs crowd the thresholds (0.6% of the voxels lie within 1e-3 of
   0.5, 6% within 1e-2; tools/bf16_diag.py), so the measured overall agreement (0.9958-0.99997 by
   threshold) is printed, not asserted at 99.9%.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def nat():
    from light_unet import _native
    return _native


def st():
    return torch.cuda.current_stream().cuda_stream


def rb(t):
    """fp32 tensor holding bf16-representable values"""
    return t.float().to(BF).float()


def ulp_key(t16):
    """monotonic integer key of bf16 values (adjacent bf16 numbers differ by 1)"""
    b = t16.contiguous().view(torch.int16).to(torch.int32)
    return torch.where(b < 0, -(b + 32768), b)


def check_act(a16, a32, what, exact_frac=0.99):
    """bf16 output vs the fp32 twin's output: <= 1 ulp after rounding, mostly exact"""
    assert a16.dtype == BF and a32.dtype == torch.float32
    r = a32.to(BF)
    assert torch.isfinite(a16.float()).all(), what
    d = (ulp_key(a16) - ulp_key(r)).abs()
    assert int(d.max()) <= 1, f"{what}: {int(d.max())} ulp"
    frac = float((d == 0).double().mean())
    assert frac >= exact_frac, f"{what}: only {frac:.4f} exact"


def check_f32(a, b, rtol, what):
    a, b = a.double().cpu(), b.double().cpu()
    scale = max(b.abs().max().item(), 1e-30)
    err = (a - b).abs().max().item() / scale
    assert err <= rtol, f"{what}: {err:.3e} > {rtol}"


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
    return rec.float()


class Twin:
    """Device copies of bf16-representable activations for both calls."""

    def __init__(self, cuda):
        self.cuda = cuda

    def act(self, t):
        t = rb(t)
        return {torch.float32: t.to(self.cuda), BF: t.to(BF).to(self.cuda)}

    def out(self, shape, fill=float("nan")):
        return {torch.float32: torch.full(shape, fill, device=self.cuda),
                BF: torch.full(shape, fill, device=self.cuda).to(BF)}

    def grad(self, t):
        """a gradient input: the same fp32 tensor for both calls"""
        t = t.float().to(self.cuda)
        return {torch.float32: t, BF: t}

    def gout(self, shape, init=None):
        """a gradient output (fp32 in both calls), optionally pre-filled (accumulate forms)"""
        return {dt: (init.float().to(self.cuda).clone() if init is not None else
                     torch.full(shape, float("nan"), device=self.cuda)) for dt in DT}


def sfx(dt):
    return "_bf16" if dt == BF else ""


def P(t):
    return None if t is None else t.data_ptr()


DT = (torch.float32, BF)

# ------------------------------------------------------------------------------ depthwise
DW_SHAPES = [(4, 16, 48, 48, 48), (4, 32, 24, 24, 24), (4, 64, 12, 12, 12), (4, 128, 6, 6, 6),
             (2, 3, 7, 6, 9), (1, 2, 4, 6, 136), (2, 4, 9, 10, 16)]


@pytest.mark.parametrize("shape", DW_SHAPES)
@pytest.mark.parametrize("mode", [0, 1])
def test_dw3_fwd_twin(cuda, shape, mode):
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(61)
    tw = Twin(cuda)
    x = tw.act(torch.randn(N, C, S, generator=gen))
    w = torch.randn(C, 27, generator=gen).to(cuda)
    rec = make_rec(N, C, gen, drop=True).to(cuda) if mode else None
    y = tw.out((N, C, S))
    for dt in DT:
        nat().call("l3u_dw3_fwd" + sfx(dt), P(x[dt]), C * S, P(w), P(rec), None, P(y[dt]), C * S,
                   N, C, D, H, W, st())
    torch.cuda.synchronize()
    check_act(y[BF], y[torch.float32], f"dw3_fwd {shape} m{mode}")


@pytest.mark.parametrize("shape", DW_SHAPES)
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_dw3_bwd_twin(cuda, shape, mode):
    """mode 0: dx = conv^T(dz); 1: IN-fused (dpre + IN sums); 2: dx += conv^T(dz)"""
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(62)
    tw = Twin(cuda)
    x, dz = tw.act(torch.randn(N, C, S, generator=gen)), tw.grad(torch.randn(N, C, S, generator=gen))
    w = torch.randn(C, 27, generator=gen).to(cuda)
    rec = make_rec(N, C, gen, drop=True).to(cuda) if mode == 1 else None
    nch = nat().query("l3u_dw3_nchunk", N, C, D, H, W)
    dx = tw.gout((N, C, S), torch.randn(N, C, S, generator=gen) if mode == 2 else None)
    dwp = {dt: torch.full((C * N * nch * 27,), float("nan"), device=cuda) for dt in DT}
    inp = {dt: torch.full((C * N * nch * 2,), float("nan"), dtype=torch.float64, device=cuda)
           for dt in DT}
    for dt in DT:
        nat().call("l3u_dw3_bwd" + sfx(dt), P(dz[dt]), C * S, P(x[dt]), C * S, P(w), P(rec),
                   P(dx[dt]), C * S, 1 if mode == 2 else 0, P(dwp[dt]),
                   P(inp[dt]) if mode == 1 else None, N, C, D, H, W, st())
    torch.cuda.synchronize()
    check_f32(dx[BF], dx[torch.float32], 1e-6, f"dw3_bwd dx {shape} m{mode}")
    check_f32(dwp[BF].view(C, -1, 27).sum(1), dwp[torch.float32].view(C, -1, 27).sum(1), 1e-5,
              f"dw3_bwd dW {shape} m{mode}")
    if mode == 1:
        check_f32(inp[BF], inp[torch.float32], 1e-5, "IN sums")


# ------------------------------------------------------------------------------ GEMMs
PW_CASES = [(4, 32, 16, 48 ** 3), (4, 16, 16, 48 ** 3), (4, 64, 32, 24 ** 3), (4, 64, 128, 12 ** 3),
            (4, 128, 128, 6 ** 3), (2, 5, 7, 37), (2, 16, 32, 1000)]


@pytest.mark.parametrize("case", PW_CASES)
def test_pw_fwd_twin(cuda, case):
    N, K, J, S = case
    gen = torch.Generator().manual_seed(63)
    tw = Twin(cuda)
    x = tw.act(torch.randn(N, K, S, generator=gen))
    w = (torch.randn(J, K, generator=gen) / K ** 0.5).to(cuda)
    b = torch.randn(J, generator=gen).to(cuda)
    y = tw.out((N, J, S))
    nsb = nat().query("l3u_pw_stat_nsb", K, J, S)
    part = {dt: torch.full((N * J * nsb * 3,), float("nan"), device=cuda) for dt in DT}
    for dt in DT:
        nat().call("l3u_pw_fwd" + sfx(dt), P(x[dt]), K * S, P(w), 0, P(b), P(y[dt]), J * S, 0,
                   P(part[dt]), N, K, J, S, st())
    torch.cuda.synchronize()
    check_act(y[BF], y[torch.float32], f"pw_fwd {case}")
    # statistics of the stored (rounded) values vs of the fp32 values
    p16, p32 = part[BF].view(N, J, nsb, 3), part[torch.float32].view(N, J, nsb, 3)
    assert torch.equal(p16[..., 0], p32[..., 0])
    check_f32(p16[..., 1], p32[..., 1], 1e-2, "block means")
    check_f32(p16[..., 2], p32[..., 2], 1e-2, "block M2")
    # accumulate form
    y0 = tw.act(torch.randn(N, J, S, generator=gen))
    for dt in DT:
        nat().call("l3u_pw_fwd" + sfx(dt), P(x[dt]), K * S, P(w), 0, None, P(y0[dt]), J * S, 1, None,
                   N, K, J, S, st())
    torch.cuda.synchronize()
    check_act(y0[BF], y0[torch.float32], f"pw_fwd acc {case}")


@pytest.mark.parametrize("case", [(4, 32, 16, 48 ** 3), (4, 64, 32, 24 ** 3), (4, 128, 64, 12 ** 3)])
def test_pw_fwd2_twin(cuda, case):
    N, K, J, S = case
    gen = torch.Generator().manual_seed(64)
    tw = Twin(cuda)
    xa, xb = tw.act(torch.randn(N, K, S, generator=gen)), tw.act(torch.randn(N, K, S, generator=gen))
    wa, wb = (torch.randn(J, K, generator=gen).to(cuda) for _ in range(2))
    ya, yb = tw.out((N, J, S)), tw.out((N, J, S))
    nsb = nat().query("l3u_pw_stat_nsb", K, J, S)
    sa = {dt: torch.empty(N * J * nsb * 3, device=cuda) for dt in DT}
    sb = {dt: torch.empty(N * J * nsb * 3, device=cuda) for dt in DT}
    for dt in DT:
        nat().call("l3u_pw_fwd2" + sfx(dt), P(xa[dt]), K * S, P(wa), P(ya[dt]), J * S, P(sa[dt]),
                   P(xb[dt]), K * S, P(wb), P(yb[dt]), J * S, P(sb[dt]), N, K, J, S, st())
    torch.cuda.synchronize()
    check_act(ya[BF], ya[torch.float32], "pw_fwd2 a")
    check_act(yb[BF], yb[torch.float32], "pw_fwd2 b")


PW_BWD_CASES = [(4, 16, 32, 48 ** 3, True), (4, 16, 16, 48 ** 3, False), (4, 32, 64, 24 ** 3, True),
                (4, 64, 32, 12 ** 3, True), (4, 128, 128, 6 ** 3, True), (2, 64, 40, 5 * 6 * 8, False)]


@pytest.mark.parametrize("case", PW_BWD_CASES)
def test_pw_bwd_twin(cuda, case):
    N, J, K, S, pro = case
    gen = torch.Generator().manual_seed(65)
    tw = Twin(cuda)
    x, dy = tw.act(torch.randn(N, K, S, generator=gen)), tw.grad(torch.randn(N, J, S, generator=gen))
    y = tw.act(torch.randn(N, J, S, generator=gen)) if pro else None
    w = (torch.randn(J, K, generator=gen) / K ** 0.5).to(cuda)
    rec = make_rec(N, J, gen).to(cuda) if pro else None
    nch = 3
    pin = (torch.randn(J, N, nch, 2, generator=gen, dtype=torch.float64) * 10).to(cuda) if pro else None
    npw = nat().query("l3u_pw_bwd_nparts", N, J, K, S)
    part = {dt: torch.full((npw * J * K,), float("nan"), device=cuda) for dt in DT}
    dx = tw.gout((N, K, S), torch.randn(N, K, S, generator=gen))
    for dt in DT:
        nat().call("l3u_pw_bwd" + sfx(dt), P(dy[dt]), J * S, P(y[dt]) if pro else None, J * S if pro else 0,
                   P(rec), P(pin), nch if pro else 0, P(x[dt]), K * S, P(w), P(dx[dt]), K * S, 1,
                   P(part[dt]), N, J, K, S, st())
    torch.cuda.synchronize()
    check_f32(dx[BF], dx[torch.float32], 1e-6, f"pw_bwd dx {case}")
    # with the IN prologue the bf16 twin rounds nothing more: identical fp32 dY
    check_f32(part[BF].view(npw, J, K).sum(0), part[torch.float32].view(npw, J, K).sum(0), 1e-5,
              f"pw_bwd dW {case}")


@pytest.mark.parametrize("case", [(4, 16, 32, 48 ** 3), (4, 32, 16, 24 ** 3), (2, 16, 8, 1000)])
def test_pw_bwd_tail_twin(cuda, case):
    N, J, K, S = case
    gen = torch.Generator().manual_seed(66)
    tw = Twin(cuda)
    out, yr = (tw.act(torch.randn(N, J, S, generator=gen)) for _ in range(2))
    dout = tw.grad(torch.randn(N, J, S, generator=gen))
    x = tw.act(torch.randn(N, K, S, generator=gen))
    w = torch.randn(J, K, generator=gen).to(cuda)
    rec = make_rec(N, J, gen).to(cuda)
    nb = 5
    tp = (torch.randn(J, N, nb, 3, generator=gen, dtype=torch.float64) * 10).to(cuda)
    npw = nat().query("l3u_pw_bwd_nparts", N, J, K, S)
    part = {dt: torch.empty(npw * J * K, device=cuda) for dt in DT}
    dx = tw.gout((N, K, S))
    for sel in (1, 2):
        for dt in DT:
            nat().call("l3u_pw_bwd_tail" + sfx(dt), P(dout[dt]), J * S, P(out[dt]), J * S, P(yr[dt]),
                       J * S, P(rec), P(tp), nb, sel, P(x[dt]), K * S, P(w), P(dx[dt]), K * S, 0,
                       P(part[dt]), N, J, K, S, st())
        torch.cuda.synchronize()
        check_f32(dx[BF], dx[torch.float32], 1e-6, f"pw_bwd_tail dx sel{sel}")
        check_f32(part[BF].view(npw, J, K).sum(0), part[torch.float32].view(npw, J, K).sum(0), 1e-5,
                  f"pw_bwd_tail dW sel{sel}")


@pytest.mark.parametrize("case", [(4, 128, 64, 6, 6, 6), (4, 64, 32, 12, 12, 12), (4, 32, 16, 24, 24, 24),
                                  (1, 8, 4, 5, 7, 9), (2, 128, 64, 16, 16, 16)])
def test_convt_twin(cuda, case):
    N, Ci, Co, D, H, W = case
    Si = D * H * W
    So = 8 * Si
    gen = torch.Generator().manual_seed(67)
    tw = Twin(cuda)
    x = tw.act(torch.randn(N, Ci, Si, generator=gen))
    w = torch.randn(Ci, Co, 8, generator=gen).to(cuda)
    b = torch.randn(Co, generator=gen).to(cuda)
    cat = tw.out((N, 2 * Co, So), 7.0)
    for dt in DT:
        nat().call("l3u_convt_fwd" + sfx(dt), P(x[dt]), Ci * Si, P(w), P(b), P(cat[dt]), 2 * Co * So,
                   N, Ci, Co, D, H, W, st())
    torch.cuda.synchronize()
    check_act(cat[BF], cat[torch.float32], f"convt fwd {case}")
    dcat = tw.grad(torch.randn(N, 2 * Co, So, generator=gen))
    for fused in (False, True):
        npf = nat().query("l3u_convt_bwd_fused_nparts", N, Ci, Co, D, H, W)
        if fused and npf == 0:
            continue
        np_ = npf if fused else nat().query("l3u_pw_bwd_weight_nparts", N, Si)
        dx = tw.gout((N, Ci, Si))
        wp = {dt: torch.empty(np_ * Ci * Co * 8, device=cuda) for dt in DT}
        bpp = {dt: torch.empty(np_ * Co, device=cuda) for dt in DT}
        name = "l3u_convt_bwd_fused" if fused else "l3u_convt_bwd"
        for dt in DT:
            nat().call(name + sfx(dt), P(dcat[dt]), 2 * Co * So, P(x[dt]), Ci * Si, P(w), P(dx[dt]),
                       Ci * Si, P(wp[dt]), P(bpp[dt]), N, Ci, Co, D, H, W, st())
        torch.cuda.synchronize()
        check_f32(dx[BF], dx[torch.float32], 1e-6, f"{name} dx {case}")
        check_f32(wp[BF].view(np_, -1).sum(0), wp[torch.float32].view(np_, -1).sum(0), 1e-5, "dW")
        check_f32(bpp[BF].view(np_, -1).sum(0), bpp[torch.float32].view(np_, -1).sum(0), 1e-5, "db")


# ------------------------------------------------------------------------------ IN tails, pool, out_conv
@pytest.mark.parametrize("shape", [(4, 16, 48, 48, 48), (4, 64, 12, 12, 12), (4, 128, 6, 6, 6),
                                   (2, 3, 5, 6, 7)])
def test_norm_act_twins(cuda, shape):
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(68)
    tw = Twin(cuda)
    y2, r = (tw.act(torch.randn(N, C, S, generator=gen)) for _ in range(2))
    dout = tw.grad(torch.randn(N, C, S, generator=gen))
    rec2, recr = make_rec(N, C, gen).to(cuda), make_rec(N, C, gen).to(cuda)
    out = tw.out((N, C, S))
    for dt in DT:
        nat().call("l3u_norm_act_fwd" + sfx(dt), P(y2[dt]), C * S, P(rec2), None, P(r[dt]), C * S,
                   P(recr), None, 1, P(out[dt]), C * S, N, C, S, st())
    torch.cuda.synchronize()
    check_act(out[BF], out[torch.float32], "norm_act_fwd")
    # backward on the bf16 block output (both twins read the same stored out)
    o = {torch.float32: out[BF].float(), BF: out[BF]}
    nb = nat().query("l3u_norm_act_nblocks", S)
    pr = {dt: torch.empty(C * N * nb * 3, dtype=torch.float64, device=cuda) for dt in DT}
    dy2, dr = tw.gout((N, C, S)), tw.gout((N, C, S))
    for dt in DT:
        nat().call("l3u_norm_act_bwd_reduce" + sfx(dt), P(dout[dt]), C * S, P(o[dt]), C * S, P(y2[dt]),
                   C * S, P(rec2), P(r[dt]), C * S, P(recr), P(pr[dt]), N, C, S, st())
        nat().call("l3u_norm_act_bwd_apply" + sfx(dt), P(dout[dt]), C * S, P(o[dt]), C * S, P(y2[dt]),
                   C * S, P(rec2), P(r[dt]), C * S, P(recr), P(pr[dt]), P(dy2[dt]), C * S, P(dr[dt]),
                   C * S, N, C, S, st())
    torch.cuda.synchronize()
    check_f32(pr[BF], pr[torch.float32], 1e-9, "tail sums")
    check_f32(dy2[BF], dy2[torch.float32], 1e-6, "norm_act_bwd dy2")
    check_f32(dr[BF], dr[torch.float32], 1e-6, "norm_act_bwd dr")
    if nb == 1:
        dy2b, drb = tw.gout((N, C, S)), tw.gout((N, C, S))
        pr1 = torch.empty(C * N * 3, dtype=torch.float64, device=cuda)
        nat().call("l3u_norm_act_bwd_bf16", P(dout[BF]), C * S, P(o[BF]), C * S, P(y2[BF]), C * S,
                   P(rec2), P(r[BF]), C * S, P(recr), P(pr1), P(dy2b[BF]), C * S, P(drb[BF]), C * S,
                   N, C, S, st())
        torch.cuda.synchronize()
        assert torch.equal(dy2b[BF], dy2[BF]) and torch.equal(drb[BF], dr[BF])
    # inner IN backward apply
    ip = (torch.randn(C, N, 3, 2, generator=gen, dtype=torch.float64) * 10).to(cuda)
    dy = tw.gout((N, C, S))
    for dt in DT:
        nat().call("l3u_in_bwd_apply" + sfx(dt), P(dout[dt]), C * S, P(y2[dt]), C * S, P(rec2), P(ip), 3,
                   P(dy[dt]), C * S, N, C, S, st())
    torch.cuda.synchronize()
    check_f32(dy[BF], dy[torch.float32], 1e-6, "in_bwd_apply")


@pytest.mark.parametrize("shape", [(4, 16, 48, 48, 48), (4, 32, 24, 24, 24), (4, 64, 12, 12, 12),
                                   (2, 3, 4, 6, 8)])
def test_norm_act_pool_and_maxpool_twins(cuda, shape):
    N, C, D, H, W = shape
    S, So = D * H * W, (D // 2) * (H // 2) * (W // 2)
    gen = torch.Generator().manual_seed(69)
    tw = Twin(cuda)
    y2, r = (tw.act(torch.randn(N, C, S, generator=gen)) for _ in range(2))
    rec2, recr = make_rec(N, C, gen).to(cuda), make_rec(N, C, gen).to(cuda)
    out, pooled = tw.out((N, C, S)), tw.out((N, C, So))
    idx = {dt: torch.empty(N * C * So, dtype=torch.uint8, device=cuda) for dt in DT}
    for dt in DT:
        nat().call("l3u_norm_act_pool_fwd" + sfx(dt), P(y2[dt]), C * S, P(rec2), None, P(r[dt]), C * S,
                   P(recr), None, 1, P(out[dt]), C * S, P(pooled[dt]), C * So, P(idx[dt]), N, C, D, H,
                   W, st())
    torch.cuda.synchronize()
    check_act(out[BF], out[torch.float32], "norm_act_pool out")
    # the bf16 pool is MaxPool3d of the stored bf16 output (monotone rounding: same maxima)
    ref = F.max_pool3d(out[BF].float().view(N, C, D, H, W), 2).view(N, C, So)
    assert torch.equal(pooled[BF].float(), ref)
    # stand-alone maxpool twin on the bf16 output, and its backward
    p2, i2 = tw.out((N, C, So)), torch.empty(N * C * So, dtype=torch.uint8, device=cuda)
    nat().call("l3u_maxpool2_fwd_bf16", P(out[BF]), C * S, P(p2[BF]), C * So, P(i2), N, C, D, H, W, st())
    torch.cuda.synchronize()
    assert torch.equal(p2[BF], pooled[BF]) and torch.equal(i2, idx[BF])
    # (the maxpool backward reads no saved activation: gradients only, fp32, no bf16 twin)


@pytest.mark.parametrize("case", [(4, 16, 48 ** 3), (2, 16, 1000), (1, 8, 37)])
def test_outconv_twin(cuda, case):
    N, C, S = case
    gen = torch.Generator().manual_seed(70)
    tw = Twin(cuda)
    h = tw.act(torch.randn(N, C, S, generator=gen))
    w = (torch.randn(C, generator=gen) * 0.3).to(cuda)
    b = torch.randn(1, generator=gen).to(cuda)
    t = (torch.rand(N, S, generator=gen) > 0.9).float().to(cuda)
    nb = nat().query("l3u_outconv_nblocks", S)
    p = {dt: torch.empty(N, S, device=cuda) for dt in DT}
    fp = {dt: torch.empty(N * nb * 3, device=cuda) for dt in DT}
    for dt in DT:
        nat().call("l3u_outconv_fwd" + sfx(dt), P(h[dt]), C * S, P(w), P(b), P(p[dt]), P(t), P(fp[dt]),
                   N, C, S, st())
    torch.cuda.synchronize()
    assert torch.equal(p[BF], p[torch.float32]) and torch.equal(fp[BF], fp[torch.float32])
    sums = torch.empty(3, dtype=torch.float64, device=cuda)
    nat().call("l3u_ftl_reduce", P(fp[BF]), N * nb, P(sums), st())
    dh = tw.gout((N, C, S))
    part = {dt: torch.empty(N * nb * (C + 1), dtype=torch.float64, device=cuda) for dt in DT}
    for dt in DT:
        nat().call("l3u_outconv_bwd" + sfx(dt), None, P(p[dt]), P(t), P(sums), 0.7, 0.3, 0.75, 1e-6, None,
                   P(h[dt]), C * S, P(w), P(dh[dt]), C * S, P(part[dt]), None, N, C, S, st())
    torch.cuda.synchronize()
    check_f32(dh[BF], dh[torch.float32], 1e-6, "outconv dh")
    assert torch.equal(part[BF], part[torch.float32])


@pytest.mark.parametrize("shape", [(4, 16, 48, 48, 48), (2, 8, 5, 6, 8)])
def test_front_twin(cuda, shape):
    N, C, D, H, W = shape
    S = D * H * W
    gen = torch.Generator().manual_seed(71)
    x = torch.randn(N, 1, S, generator=gen).to(cuda)   # the caller's fp32 input
    wdw, w1, wr = (torch.randn(n, generator=gen).to(cuda) for n in (27, C, C))
    tw = Twin(cuda)
    z1, y1, r, xc = tw.out((N, 1, S)), tw.out((N, C, S)), tw.out((N, C, S)), tw.out((N, 1, S))
    nb = nat().query("l3u_front_nblocks", S)
    s1 = {dt: torch.empty(N * C * nb * 3, device=cuda) for dt in DT}
    sr = {dt: torch.empty(N * C * nb * 3, device=cuda) for dt in DT}
    for dt in DT:
        nat().call("l3u_front_fwd" + sfx(dt), P(x), S, P(wdw), P(w1), P(wr), P(z1[dt]), P(y1[dt]),
                   P(r[dt]), P(s1[dt]), P(sr[dt]), P(xc[dt]) if dt == BF else None, N, C, D, H, W, st())
    torch.cuda.synchronize()
    for a in (z1, y1, r):
        check_act(a[BF], a[torch.float32], "front")
    assert torch.equal(xc[BF], x.to(BF))
    assert torch.equal(s1[BF], s1[torch.float32]) and torch.equal(sr[BF], sr[torch.float32])


def test_casts(cuda):
    gen = torch.Generator().manual_seed(72)
    x = torch.randn(1001, generator=gen).to(cuda)
    y = torch.empty(1001, dtype=BF, device=cuda)
    z = torch.empty(1001, device=cuda)
    nat().call("l3u_cast_f32_bf16", P(x), P(y), 1001, st())
    nat().call("l3u_cast_bf16_f32", P(y), P(z), 1001, st())
    torch.cuda.synchronize()
    assert torch.equal(y, x.to(BF)) and torch.equal(z, y.float())


# ------------------------------------------------------------------------------ the network
def _model(z, cuda, **kw):
    from light_unet.models.unet3d import Lightweight3DUNet
    m = Lightweight3DUNet(dropout_p=0.0, **kw)
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")})
    return m.to(cuda).train()


def _run(model, z, cuda):
    from light_unet.models.losses import FocalTverskyLoss
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)
    out = model(x)
    loss = FocalTverskyLoss()(out, t)
    model.zero_grad(set_to_none=True)
    loss.backward()
    torch.cuda.synchronize()
    g = {k: p.grad.detach().cpu().double().numpy() for k, p in model.named_parameters()}
    return out.detach().cpu().numpy(), float(loss), g


@pytest.mark.parametrize("fname", ["model_b2_32.npz", "model_b1_48.npz"])
def test_bf16_model_vs_golden_and_fp32(cuda, golden, fname):
    z = golden(fname)
    o16, l16, g16 = _run(_model(z, cuda, compute_dtype=BF), z, cuda)
    o32, l32, g32 = _run(_model(z, cuda), z, cuda)
    ref = z["out"]
    assert o16.dtype == np.float32
    err = np.abs(o16 - ref).max()
    assert err <= 2e-2, err
    assert np.abs(o16 - o32).max() <= 2e-2
    agrees = []
    for thr in (0.1, 0.3, 0.5, 0.7):
        m16, mref = o16 >= thr, ref >= thr
        far = np.abs(ref - thr) > 2e-2
        assert np.array_equal(m16[far], mref[far]), thr
        agree = float(np.mean(m16 == mref))
        assert agree >= 0.995, (thr, agree)
        agrees.append(agree)
    lr = float(z["loss"])
    assert abs(l16 - lr) <= 1e-2 * abs(lr), (l16, lr)
    num = sum(np.sum((g16[k] - z["g/" + k]) ** 2) for k in g16)
    den = sum(np.sum(z["g/" + k].astype(np.float64) ** 2) for k in g16)
    gerr = (num / den) ** 0.5
    num32 = sum(np.sum((g32[k] - z["g/" + k]) ** 2) for k in g32)
    print(f"bf16 {fname}: out err {err:.2e}, loss {l16:.6f} vs {lr:.6f}, grad rel L2 {gerr:.2e} "
          f"(fp32 HIP {(num32 / den) ** 0.5:.2e}), mask agreement {agrees}")
    dot = sum(np.sum(g16[k] * z["g/" + k]) for k in g16)
    n16 = sum(np.sum(g16[k] ** 2) for k in g16)
    cos = dot / (n16 * den) ** 0.5
    print(f"   gradient cosine to the fp64 golden {cos:.5f}")
    assert gerr <= 0.2 and cos >= 0.98, (gerr, cos)


def test_bf16_autocast_selects_the_bf16_path(cuda, golden):
    """torch.autocast("cuda", dtype=torch.bfloat16) runs the same bf16 kernels as
    compute_dtype=torch.bfloat16 (bitwise); outside autocast the model is fp32."""
    z = golden("model_b2_32.npz")
    x = torch.from_numpy(z["x"]).to(cuda)
    m = _model(z, cuda).eval()
    mb = _model(z, cuda, compute_dtype=BF).eval()
    with torch.no_grad():
        with torch.autocast("cuda", dtype=BF):
            pa = m(x)
        pb = mb(x)
        p32 = m(x)
    assert torch.equal(pa, pb)
    assert not torch.equal(p32, pb) and (p32 - pb).abs().max().item() <= 2e-2


def test_bf16_trainstep_graph_equals_eager_and_tracks_fp32(cuda, golden):
    """TrainStep(dtype=bf16): hipGraph replay == eager (bitwise); over 4 steps the bf16 losses
    follow the fp32 step's within 1e-2 relative (fp32 master weights and AdamW)."""
    from light_unet.train_step import TrainStep
    z = golden("model_b2_32.npz")
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)
    steps = 4
    la = [TrainStep(_model(z, cuda), dtype=torch.float32)(x, t).item() for _ in range(1)]
    ts32 = TrainStep(_model(z, cuda))
    l32 = [ts32(x, t).item() for _ in range(steps)]
    ts16 = TrainStep(_model(z, cuda), dtype=BF)
    l16 = [ts16(x, t).item() for _ in range(steps)]
    tg = TrainStep(_model(z, cuda), dtype=BF)
    xs, tsb = x.clone(), t.clone()
    tg.capture(xs, tsb)
    lg = [tg.replay().item() for _ in range(steps)]
    assert la[0] == l32[0]
    np.testing.assert_allclose(l16, l32, rtol=1e-2)
    assert l16 == lg
    assert torch.equal(ts16.flat, tg.flat)


def _stored(model, x):
    """The bf16 engine's stored activations of one forward, keyed as oracle/bf16_oracle.Storage
    expects: <block> + z1 / y1 / r / z2 / y2 / out, <up> + u (the ConvTranspose3d output, the lower
    half of the concat buffer)."""
    eng = model.engine
    eng.set_act_dtype(BF)
    _, sv = eng.forward(model.flat_parameters(), x, training=True, dropout_p=0.0, save=True)
    torch.cuda.synchronize()
    return _stored_sv(sv, x.shape[0])


def _stored_sv(sv, N):
    """_stored from a forward's saved state (the engine's own, or a TrainStep's)."""
    out = {}
    for pre, b in sv["blk"].items():
        d, h, w = b["dims"]
        S = d * h * w
        for key in ("z1", "y1", "z2", "y2"):
            out[pre + key] = b[key].double().cpu()
        for key in ("r", "out", "x"):
            v = b.get(key)
            if v is None:
                continue
            flat = v.t.reshape(-1)
            t = torch.stack([flat[n * v.ns + v.off: n * v.ns + v.off + v.C * S] for n in range(N)])
            out[pre + key] = t.double().cpu().reshape(N, v.C, d, h, w)
    for up in ("up1.", "up2.", "up3."):
        cat = out.pop(up + "res_block.x")
        out[up + "u"] = cat[:, :cat.shape[1] // 2]
    return {k: v for k, v in out.items() if not k.endswith(".x")}


@pytest.mark.parametrize("fname", ["model_b2_32.npz", "model_b1_48.npz"])
def test_bf16_model_vs_bf16_storage_oracle(cuda, golden, fname):
    """The HIP bf16 network against oracle/bf16_oracle.py, the reference network (fp64) with bf16
    rounding exactly where the engine stores activations, driven by the engine's own stored
    tensors (teacher forcing: each storage point takes the engine's value forward and passes the
    gradient straight through).  Free-running, the two chains cannot agree elementwise: a bf16
    tie decided differently by fp32 and fp64 arithmetic moves one stored value by one ulp, and the
    next rounding amplifies it (measured: 6.5e-2 gradient rel L2 apart, against 0.13 from the fp64
    golden).  Forced, every op of the chain is checked on the engine's own inputs:
      * each stored tensor is R(op(stored inputs)): at most 1e-3 of its elements differ, each
        by <= 1 bf16 ulp or by <= 1e-6 of the tensor's max (fp32 cancellation in near-zero sums);
      * output |diff| <= 1e-5, loss 1e-6 relative, whole-gradient rel L2 <= 1e-3 (the backward is
        the gradient of the bf16-storage forward the engine computed)."""
    from oracle import bf16_oracle as B16
    from oracle import unet_oracle as U
    z = golden(fname)
    m = _model(z, cuda, compute_dtype=BF)
    x = torch.from_numpy(z["x"]).to(cuda)
    stored = _stored(m, x)
    o16, l16, g16 = _run(m, z, cuda)
    sd = {k[2:]: torch.from_numpy(z[k]).double().requires_grad_(True) for k in z.files if k.startswith("w/")}
    st = B16.Storage(stored)
    pb = B16.unet_forward(sd, torch.from_numpy(z["x"]).double(), st=st)
    lb = U.focal_tversky(pb, torch.from_numpy(z["target"]).double())
    lb.backward()
    assert set(st.pairs) == set(stored), set(stored) ^ set(st.pairs)
    worst = 0.0
    for k, (r, e) in st.pairs.items():
        ulp = (r.to(BF).view(torch.int16).long() - e.to(BF).view(torch.int16).long()).abs()
        near = (r - e).abs() <= 1e-6 * r.abs().max()
        assert bool(((ulp <= 1) | near).all()), (k, int(ulp.max()))
        frac = float((r != e).double().mean())
        worst = max(worst, frac)
        assert frac <= 1e-3, (k, frac)
    oerr = float(np.abs(o16 - pb.detach().numpy()).max())
    gb = {k: v.grad.numpy() for k, v in sd.items()}
    num = sum(np.sum((g16[k] - gb[k]) ** 2) for k in gb)
    den = sum(np.sum(gb[k] ** 2) for k in gb)
    gerr = (num / den) ** 0.5
    print(f"bf16 {fname} vs bf16-storage oracle (forced): {len(st.pairs)} storage points, worst "
          f"mismatch fraction {worst:.1e}; out {oerr:.1e}, loss {l16:.7f} vs {lb.item():.7f}, "
          f"grad rel L2 {gerr:.1e}")
    assert oerr <= 1e-5, oerr
    assert abs(l16 - lb.item()) <= 1e-6 * abs(lb.item())
    assert gerr <= 1e-3, gerr


@pytest.mark.timeout(300)
def test_bf16_trainstep_bs4_48_vs_bf16_storage_oracle(cuda):
    """BASELINE config 3's step at the benchmarked shape: the product TrainStep(dtype=bf16) at
    bs 4 x 48^3 (bench.py's `bf16` leg), eager and hipGraph-replayed, against the bf16-storage
    oracle driven by the step's own stored tensors (the bounds of
    test_bf16_model_vs_bf16_storage_oracle: every stored tensor within 1 bf16 ulp of the op on the
    engine's inputs on >= 99.9% of its elements, output 1e-5, loss 1e-6 relative, whole-gradient
    relative L2 1e-3); the replayed step equals the eager one bitwise."""
    from oracle import bf16_oracle as B16
    from oracle import unet_oracle as U
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    torch.manual_seed(42)
    model = Lightweight3DUNet(dropout_p=0.0)
    sd0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
    rng = np.random.default_rng(42)
    xh = torch.from_numpy(rng.random((4, 1, 48, 48, 48), dtype=np.float32))
    th = torch.from_numpy((rng.random((4, 1, 48, 48, 48)) > 0.97).astype(np.float32))
    x, t = xh.to(cuda), th.to(cuda)
    m = model.to(cuda).train()
    ts = TrainStep(m, dtype=BF)
    p, sv, sums = ts._fwd(x, t)
    torch.cuda.synchronize()
    stored = _stored_sv(sv, 4)
    ts._bwd(p, sv, t, sums)
    torch.cuda.synchronize()
    o16 = p.detach().cpu().numpy()
    l16 = float(ts.loss.item())
    gflat = ts.gflat.clone()
    del p, sv, sums
    # the replayed step
    m2 = Lightweight3DUNet(dropout_p=0.0)
    m2.load_state_dict(sd0)
    tg = TrainStep(m2.to(cuda).train(), dtype=BF)
    xs, tsb = x.clone(), t.clone()
    tg.capture(xs, tsb)
    assert float(tg.replay().item()) == l16
    torch.cuda.synchronize()
    assert torch.equal(tg.gflat, gflat) and torch.equal(tg.flat, ts.flat)
    del tg, m2
    g = gflat.cpu().double().numpy()
    g16 = {k: g[o:o + n].reshape(shape) for k, (o, n, shape) in m.engine.offsets.items()}
    sd = {k: v.double().requires_grad_(True) for k, v in sd0.items()}
    st = B16.Storage(stored)
    pb = B16.unet_forward(sd, xh.double(), st=st)
    lb = U.focal_tversky(pb, th.double())
    lb.backward()
    assert set(st.pairs) == set(stored), set(stored) ^ set(st.pairs)
    worst = 0.0
    for k, (r, e) in st.pairs.items():
        ulp = (r.to(BF).view(torch.int16).long() - e.to(BF).view(torch.int16).long()).abs()
        near = (r - e).abs() <= 1e-6 * r.abs().max()
        assert bool(((ulp <= 1) | near).all()), (k, int(ulp.max()))
        frac = float((r != e).double().mean())
        worst = max(worst, frac)
        assert frac <= 1e-3, (k, frac)
    oerr = float(np.abs(o16 - pb.detach().numpy()).max())
    gb = {k: v.grad.numpy() for k, v in sd.items()}
    num = sum(np.sum((g16[k] - gb[k]) ** 2) for k in gb)
    den = sum(np.sum(gb[k] ** 2) for k in gb)
    gerr = (num / den) ** 0.5
    print(f"bf16 TrainStep bs 4 x 48^3 vs bf16-storage oracle (forced): {len(st.pairs)} storage "
          f"points, worst mismatch fraction {worst:.1e}; out {oerr:.1e}, loss {l16:.7f} vs "
          f"{lb.item():.7f}, grad rel L2 {gerr:.1e}")
    assert oerr <= 1e-5, oerr
    assert abs(l16 - lb.item()) <= 1e-6 * abs(lb.item())
    assert gerr <= 1e-3, gerr
