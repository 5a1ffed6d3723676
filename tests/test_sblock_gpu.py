"""l3u_sblock_fwd: the one-launch ResidualBlock forward at small volumes (unet3d.py:77-93 with
DepthwiseSeparableConv3d convs, :10-23) against an fp64 torch restatement of the same block, every
saved intermediate included, and the whole network with the fused block against the level-by-level
schedule (the default; the fused block is opt-in, L3U_SBLOCK=1).

Tolerances: z1 / y1 / r / z2 / y2 / out are <= 27- or K-term fp32 sums of O(1) operands: 2e-5 of
the tensor max against fp64 (bf16 storage: 2e-2).  Records: mean / rstd 1e-5 relative.  The
network with and without the fused block differs only in fp32 summation order: output 1e-5,
loss 1e-5 relative, gradients 1e-4 (global relative L2)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from test_ops_gpu import close, nat, st

pytestmark = pytest.mark.gpu

SLOPE = 0.01

# (N, Cin, Cout, D, H, W, shortcut): down3 and bottleneck of the shipped 48^3 / 32^3 network, the
# ragged 5x5x4 bottom level of a 40x44x36 patch, a one-group block, a 256-voxel volume
SHAPES = [(4, 64, 128, 6, 6, 6, 1), (4, 128, 128, 6, 6, 6, 0), (2, 32, 64, 5, 5, 4, 1),
          (1, 16, 16, 3, 4, 5, 0), (2, 64, 64, 4, 8, 8, 0), (3, 16, 32, 6, 6, 6, 1)]


def _inorm(y, g, b):
    m = y.mean(dim=(2, 3, 4), keepdim=True)
    v = y.var(dim=(2, 3, 4), unbiased=False, keepdim=True)
    return (y - m) / torch.sqrt(v + 1e-5) * g[None, :, None, None, None] + b[None, :, None, None, None]


def _args(N, Cin, Cout, S, sc, dt, cuda, gen, drop):
    def r(*s, scale=1.0):
        return (torch.randn(*s, generator=gen, dtype=torch.float64) * scale)
    P = {"x": r(N, Cin, S), "wdw1": r(Cin, 27, scale=0.3), "wpw1": r(Cout, Cin, scale=Cin ** -0.5),
         "wdw2": r(Cout, 27, scale=0.3), "wpw2": r(Cout, Cout, scale=Cout ** -0.5),
         "g1": 1 + 0.2 * r(Cout), "b1": 0.2 * r(Cout), "g2": 1 + 0.2 * r(Cout), "b2": 0.2 * r(Cout)}
    if sc:
        P.update(wsc=r(Cout, Cin, scale=Cin ** -0.5), gsc=1 + 0.2 * r(Cout), bsc=0.2 * r(Cout))
    D = {k: v.float().to(cuda) for k, v in P.items()}
    D["x"] = D["x"].to(dt)
    out = {k: torch.full(s, float("nan"), device=cuda).to(dt) for k, s in
           (("z1", (N, Cin, S)), ("y1", (N, Cout, S)), ("z2", (N, Cout, S)), ("y2", (N, Cout, S)),
            ("r", (N, Cout, S)), ("out", (N, Cout, S)))}
    recs = torch.full((3, N, Cout, 8), float("nan"), device=cuda)
    sync = torch.zeros(N + 1, dtype=torch.int32, device=cuda)
    step = torch.tensor([7], dtype=torch.int32, device=cuda)
    p = lambda k: D[k].data_ptr() if k in D else None  # noqa: E731
    a = nat().SblockFwdArgs(
        D["x"].data_ptr(), Cin * S, p("wdw1"), p("wpw1"), p("wsc"), p("gsc"), p("bsc"), p("g1"),
        p("b1"), p("wdw2"), p("wpw2"), p("g2"), p("b2"), drop, 3, 0x1234, step.data_ptr(),
        out["z1"].data_ptr(), out["y1"].data_ptr(), out["z2"].data_ptr(), out["y2"].data_ptr(),
        out["r"].data_ptr() if sc else None, out["out"].data_ptr(), Cout * S,
        recs[0].data_ptr() if sc else None, recs[1].data_ptr(), recs[2].data_ptr(), sync.data_ptr())
    return P, D, out, recs, sync, step, a


@pytest.mark.parametrize("shape", SHAPES)
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_sblock_matches_fp64_block(cuda, shape, dt):
    import ctypes
    N, Cin, Cout, Dd, H, W, sc = shape
    if not nat().query("l3u_sblock_supported", N, Cin, Cout, Dd, H, W, sc):
        pytest.skip("shape outside the fused kernel")
    S = Dd * H * W
    drop = 0.25
    gen = torch.Generator().manual_seed(71)
    P, Dv, out, recs, sync, _, a = _args(N, Cin, Cout, S, sc, dt, cuda, gen, drop)
    sfx = "_bf16" if dt == torch.bfloat16 else ""
    nat().call("l3u_sblock_fwd" + sfx, ctypes.pointer(a), N, Cin, Cout, Dd, H, W, st())
    torch.cuda.synchronize()
    assert sync[N].item() == 0, "a sample barrier timed out"
    assert (sync[:N] == 2 * (Cout // 16)).all()
    # fp64 restatement (bf16: from the bf16-rounded input, as the kernel sees it)
    x = Dv["x"].double().cpu().view(N, Cin, Dd, H, W)
    z1 = F.conv3d(x, P["wdw1"].view(Cin, 1, 3, 3, 3), padding=1, groups=Cin)
    y1 = F.conv3d(z1, P["wpw1"].view(Cout, Cin, 1, 1, 1))
    keep = recs[1, :, :, 4].double().cpu()                     # the kernel's Dropout3d draw
    kv = keep.numpy()
    assert np.all((kv == 0) | (np.abs(kv - 1.0 / (1.0 - drop)) < 1e-6))
    a1 = F.leaky_relu(_inorm(y1, P["g1"], P["b1"]), SLOPE) * keep[:, :, None, None, None]
    z2 = F.conv3d(a1, P["wdw2"].view(Cout, 1, 3, 3, 3), padding=1, groups=Cout)
    y2 = F.conv3d(z2, P["wpw2"].view(Cout, Cout, 1, 1, 1))
    if sc:
        r = F.conv3d(x, P["wsc"].view(Cout, Cin, 1, 1, 1))
        res = _inorm(r, P["gsc"], P["bsc"])
    else:
        res = x
    o = F.leaky_relu(_inorm(y2, P["g2"], P["b2"]) + res, SLOPE)
    tol = 2e-5 if dt == torch.float32 else 3e-2
    for name, ref in (("z1", z1), ("y1", y1), ("z2", z2), ("y2", y2), ("out", o)) + \
            ((("r", r),) if sc else ()):
        close(out[name].view_as(ref), ref, tol, f"{name} {shape} {dt}")
    # records: mean / rstd of y1 and y2 (of the stored values), affine parameters
    for k, y, g, b in ((1, y1, P["g1"], P["b1"]), (2, y2, P["g2"], P["b2"])):
        rc = recs[k].double().cpu()
        ys = out["y1" if k == 1 else "y2"].double().cpu().view(N, Cout, S)
        close(rc[..., 0], ys.mean(-1), 1e-5, f"rec{k} mean")
        close(rc[..., 1], 1 / torch.sqrt(ys.var(-1, unbiased=False) + 1e-5), 1e-5, f"rec{k} rstd")
        close(rc[..., 5], g.expand(N, Cout), 1e-6, f"rec{k} gamma")
    assert torch.equal(recs[2, :, :, 4].cpu(), torch.ones(N, Cout))   # no dropout after norm2
    if drop > 0 and N * Cout >= 64:
        assert (keep == 0).any() and (keep > 0).any()


def test_sblock_repeat_launches_identical(cuda):
    """The barrier counters are never reset: 40 back-to-back launches on one counter array give
    the same bits as the first (and the counters advance by 2 episodes per launch)."""
    import ctypes
    N, Cin, Cout, Dd, H, W, sc = SHAPES[0]
    S = Dd * H * W
    gen = torch.Generator().manual_seed(72)
    _, _, out, recs, sync, step, a = _args(N, Cin, Cout, S, sc, torch.float32, cuda, gen, 0.1)
    nat().call("l3u_sblock_fwd", ctypes.pointer(a), N, Cin, Cout, Dd, H, W, st())
    torch.cuda.synchronize()
    first = {k: v.clone() for k, v in out.items()}
    for _ in range(40):
        nat().call("l3u_sblock_fwd", ctypes.pointer(a), N, Cin, Cout, Dd, H, W, st())
    torch.cuda.synchronize()
    assert sync[N].item() == 0
    assert (sync[:N] == 41 * 2 * (Cout // 16)).all()
    for k, v in out.items():
        assert torch.equal(v, first[k]), k


def test_sblock_rejects_unsupported(cuda):
    # more workgroups than compute units, Cout not a multiple of 16, a volume above 256 voxels
    assert not nat().query("l3u_sblock_supported", 4096, 128, 128, 6, 6, 6, 0)
    assert not nat().query("l3u_sblock_supported", 4, 24, 24, 6, 6, 6, 0)
    assert not nat().query("l3u_sblock_supported", 4, 64, 64, 7, 7, 7, 0)
    assert nat().query("l3u_sblock_supported", 4, 64, 128, 6, 6, 6, 1)


@pytest.mark.parametrize("fixture", ["model_b1_48.npz", "model_b2_32.npz", "model_b1_40_44_36.npz"])
def test_network_with_sblock_matches_level_schedule(cuda, golden, fixture):
    """Train-mode step (Dropout3d 0.1) with the fused small-volume blocks vs L3U_SBLOCK=0: same
    masks (same stream ids), outputs / loss / every parameter gradient to fp32 summation order."""
    import light_unet.engine as E
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    z = golden(fixture)
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)
    res = []
    keep = E._SBLOCK
    for on in (True, False):
        E._SBLOCK = on
        try:
            m = Lightweight3DUNet(dropout_p=0.1)
            m.load_state_dict(sd)
            m = m.to(cuda).train()
            ts = TrainStep(m)
            p, sv, sums = ts._fwd(x, t)
            ts._bwd(p, sv, t, sums)
            torch.cuda.synchronize()
            res.append((p.clone(), ts.loss.clone(), ts.gflat.clone(),
                        {k: b["recs"][1][:, 4].clone() for k, b in sv["blk"].items()}))
        finally:
            E._SBLOCK = keep
    (p1, l1, g1, k1), (p0, l0, g0, k0) = res
    for k in k1:
        assert torch.equal(k1[k], k0[k]), f"dropout masks differ in {k}"
    assert (p1 - p0).abs().max().item() <= 1e-5
    assert abs(l1.item() - l0.item()) <= 1e-5 * abs(l0.item())
    rel = ((g1 - g0).double().norm() / g0.double().norm()).item()
    assert rel <= 1e-4, rel
