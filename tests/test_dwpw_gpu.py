"""l3u_dwpw_fwd: the fused depthwise-separable conv forward (DepthwiseSeparableConv3d.forward,
light_unet/models/unet3d.py:20-23, plus the block's Conv1x1 shortcut :70-73) against the unfused
C-ABI pair l3u_dw3_fwd -> l3u_pw_fwd (/ l3u_pw_fwd2) on the same inputs, and its InstanceNorm
partials against torch statistics.  Tolerances: Z and Y equal the unfused kernels to fp32 rounding
(1e-6 of the tensor max; the tap and k orders are the same); statistics 1e-5."""
import pytest
import torch

from test_ops_gpu import close, make_rec, nat, st

pytestmark = pytest.mark.gpu

# (N, K, Nout, D, H, W, shortcut, xf): the model's 48^3 conv2 (16 -> 16, IN on load), the 24^3
# down1.conv1 (16 -> 32 with the shortcut), a ragged volume (short last strip and slab)
# (the 48^3 shortcut form exercises the four-slot plane ring of the one-step-late shortcut GEMM)
SHAPES = [(4, 16, 16, 48, 48, 48, 0, 1), (2, 16, 32, 24, 24, 24, 1, 0), (4, 16, 16, 48, 48, 48, 1, 0),
          (1, 16, 16, 20, 28, 36, 0, 1), (2, 16, 32, 13, 10, 12, 0, 1), (1, 16, 32, 9, 7, 16, 0, 0)]


def _merge(part):
    """(count, mean, M2) partials [N][C][nsb][3] -> mean, biased variance (fp64, host)."""
    p = part.double().cpu()
    c, m, m2 = p[..., 0], p[..., 1], p[..., 2]
    n = c.sum(-1)
    mean = (c * m).sum(-1) / n
    M2 = m2.sum(-1) + (c * (m - mean[..., None]) ** 2).sum(-1)
    return mean, M2 / n


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_dwpw_equals_unfused(cuda, shape, dt):
    N, K, J, D, H, W, sc, xf = shape
    if not nat().query("l3u_dwpw_supported", K, J, D, H, W, sc):
        pytest.skip("shape outside the fused kernel")
    sfx = "_bf16" if dt == torch.bfloat16 else ""
    S = D * H * W
    gen = torch.Generator().manual_seed(61)
    xfull = torch.randn(N, 2 * K, S, generator=gen).to(cuda).to(dt)   # upper half of a concat
    x = xfull[:, K:]
    wdw = (torch.randn(K, 27, generator=gen) * 0.3).to(cuda)
    wpw = torch.randn(J, K, generator=gen).to(cuda)
    wsc = torch.randn(J, K, generator=gen).to(cuda) if sc else None
    rec = make_rec(N, K, gen, drop=True).float().to(cuda) if xf else None
    nsb = nat().query("l3u_dwpw_stat_nsb", K, J, D, H, W)

    def e(*s):
        return torch.full(s, float("nan"), device=cuda).to(dt)
    y, z, r = e(N, J, S), e(N, K, S), e(N, J, S)
    ys = torch.full((N * J * nsb * 3,), float("nan"), device=cuda)
    rs = torch.full((N * J * nsb * 3,), float("nan"), device=cuda)
    nat().call("l3u_dwpw_fwd" + sfx, x.data_ptr(), 2 * K * S, wdw.data_ptr(),
               rec.data_ptr() if xf else None, None, wpw.data_ptr(), y.data_ptr(), J * S,
               ys.data_ptr(), wsc.data_ptr() if sc else None, r.data_ptr() if sc else None, J * S,
               rs.data_ptr() if sc else None, z.data_ptr(), K * S, N, K, J, D, H, W, st())
    # the unfused pair
    z0, y0, r0 = e(N, K, S), e(N, J, S), e(N, J, S)
    nat().call("l3u_dw3_fwd" + sfx, x.data_ptr(), 2 * K * S, wdw.data_ptr(),
               rec.data_ptr() if xf else None, None, z0.data_ptr(), K * S, N, K, D, H, W, st())
    nat().call("l3u_pw_fwd" + sfx, z0.data_ptr(), K * S, wpw.data_ptr(), 0, None, y0.data_ptr(), J * S,
               0, None, N, K, J, S, st())
    if sc:
        nat().call("l3u_pw_fwd" + sfx, x.data_ptr(), 2 * K * S, wsc.data_ptr(), 0, None, r0.data_ptr(),
                   J * S, 0, None, N, K, J, S, st())
    torch.cuda.synchronize()
    tol = 1e-6 if dt == torch.float32 else 1e-2
    close(z, z0, tol, "Z")
    close(y, y0, tol, "Y")
    if sc:
        close(r, r0, tol, "R")
    for out, part in ((y, ys), (r, rs)) if sc else ((y, ys),):
        mean, var = _merge(part.view(N, J, nsb, 3))
        o = out.double().cpu()
        close(mean, o.mean(-1), 1e-5, "IN mean")
        close(var, o.var(-1, unbiased=False), 1e-5, "IN var")


def test_dwpw_record_in_kernel(cuda):
    """conv2 with the InstanceNorm record finalized in-kernel from the conv1 partials (src) equals
    the call with that record precomputed by l3u_in_finalize; rec_out is the same record."""
    N, K, J, D, H, W = 2, 16, 16, 16, 24, 24
    S = D * H * W
    gen = torch.Generator().manual_seed(62)
    x = torch.randn(N, K, S, generator=gen).to(cuda)
    wdw = (torch.randn(K, 27, generator=gen) * 0.3).to(cuda)
    wpw = torch.randn(K, K, generator=gen).to(cuda)
    nsb = nat().query("l3u_dwpw_stat_nsb", K, K, D, H, W)
    y1 = torch.empty(N, K, S, device=cuda)
    p1 = torch.empty(N * K * nsb * 3, device=cuda)
    nat().call("l3u_dwpw_fwd", x.data_ptr(), K * S, wdw.data_ptr(), None, None, wpw.data_ptr(),
               y1.data_ptr(), K * S, p1.data_ptr(), None, None, 0, None, None, 0, N, K, K, D, H, W,
               st())
    g = (1 + 0.1 * torch.randn(K, generator=gen)).to(cuda)
    b = (0.1 * torch.randn(K, generator=gen)).to(cuda)
    step = torch.tensor([3], dtype=torch.int32, device=cuda)
    rec = torch.empty(N * K * 8, device=cuda)
    nat().call("l3u_in_finalize", p1.data_ptr(), nsb, g.data_ptr(), b.data_ptr(), 0.25, 77,
               step.data_ptr(), 2, rec.data_ptr(), N, K, st())
    rec_out = torch.full((N * K * 8,), float("nan"), device=cuda)
    src = nat().NormSrc(p1.data_ptr(), nsb, 2, g.data_ptr(), b.data_ptr(), 0.25, 77, step.data_ptr(),
                        rec_out.data_ptr())
    ya, yb = torch.empty(N, J, S, device=cuda), torch.empty(N, J, S, device=cuda)
    nat().call("l3u_dwpw_fwd", y1.data_ptr(), K * S, wdw.data_ptr(), None, nat().norm_src_ptr(src),
               wpw.data_ptr(), ya.data_ptr(), J * S, None, None, None, 0, None, None, 0, N, K, J, D,
               H, W, st())
    nat().call("l3u_dwpw_fwd", y1.data_ptr(), K * S, wdw.data_ptr(), rec.data_ptr(), None,
               wpw.data_ptr(), yb.data_ptr(), J * S, None, None, None, 0, None, None, 0, N, K, J, D,
               H, W, st())
    torch.cuda.synchronize()
    assert torch.equal(rec_out, rec)
    assert torch.equal(ya, yb)
    # and the record is the torch InstanceNorm statistics of y1
    r = rec.view(N, K, 8).double().cpu()
    yy = y1.double().cpu()
    close(r[..., 0], yy.mean(-1), 1e-5, "mean")
    close(r[..., 1], 1 / torch.sqrt(yy.var(-1, unbiased=False) + 1e-5), 1e-5, "rstd")
