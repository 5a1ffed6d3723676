"""Whole-network parity of the MI355X path against the golden fixtures made by the REFERENCE
(tests/golden/make_goldens.py imports /root/reference by file path, fp64) and against the oracle.

Tolerances (written here, as the north star asks):
  * output probabilities: |HIP - golden| <= 1e-3 absolute (north star: 1e-3 fp32); observed ~1e-6.
  * loss: |HIP - golden| <= 1e-4 relative.
  * parameter gradients: the relative L2 error of the whole gradient vector (217,228 entries) vs
    the fp64 golden must be <= max(1e-3, 2 * e32), e32 being the same error of the fp32 CPU
    oracle (torch aten = the reference's own fp32 arithmetic) on the same inputs, and every
    tensor's relative L2 error <= max(1e-2, 3 * its e32).  Why not an elementwise bound: at 48^3
    about 1-4 of the 1.77M InstanceNorm outputs of a block lie within 1e-6 of the LeakyReLU kink,
    and fp32 rounding (any fp32 implementation, the reference's included) decides which branch
    they take; each flip changes that voxel's gradient 100x and spreads through the backward
    convolutions (measured: HIP global error 7.6e-4 vs 1.1e-3 for CPU fp32 at 48^3; both 1.4e-5 at
    32^3, tools/diag_model.py).  Scale-invariant tensors (1-channel conv -> InstanceNorm, e.g.
    init_conv.shortcut.0.weight) have a true gradient ~0, which the e32 term absorbs.
  * thresholded masks (p >= thr): bit-exact on every voxel farther than 1e-4 from the threshold.
"""
import numpy as np
import pytest
import torch

from oracle import unet_oracle as U

pytestmark = pytest.mark.gpu


def _model(z, enc, cuda, dropout_p=0.0):
    from light_unet.models.unet3d import Lightweight3DUNet
    m = Lightweight3DUNet(encoder_channels=list(enc), dropout_p=dropout_p)
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    m.load_state_dict(sd)
    return m.to(cuda), sd


def _grad_errs(grads, z):
    """per-tensor relative L2 errors and the global relative L2 error vs the fp64 golden"""
    errs, num, den = {}, 0.0, 0.0
    for k, g in grads.items():
        gr = z["g/" + k].astype(np.float64)
        d = np.linalg.norm(g.astype(np.float64) - gr)
        errs[k] = d / max(np.linalg.norm(gr), 1e-30)
        num += d * d
        den += float(np.sum(gr * gr))
    return errs, (num / den) ** 0.5


def _cpu_fp32_errs(sd, z):
    params = {k: v.clone().float().requires_grad_(True) for k, v in sd.items()}
    out = U.unet_forward(params, torch.from_numpy(z["x"]))
    loss = U.focal_tversky(out, torch.from_numpy(z["target"]))
    loss.backward()
    return _grad_errs({k: p.grad.numpy() for k, p in params.items()}, z)


# (fixture, encoder channels): bs 2 at 32^3, bs 1 at 48^3, the config-5 network (32 -> 256,
# 812,284 parameters) at 64^3, a ragged volume (40 x 44 x 36: the UpBlock pad branch,
# unet3d.py:130-138, at every decoder level; odd pooled sizes 11, 5, 9, 4) and large planes (80 x 80)
GOLDEN_MODELS = [("model_b2_32.npz", (16, 32, 64, 128)), ("model_b1_48.npz", (16, 32, 64, 128)),
                 ("model_c32_b1_64.npz", (32, 64, 128, 256)),
                 ("model_b1_40_44_36.npz", (16, 32, 64, 128)),
                 ("model_b1_24_80_80.npz", (16, 32, 64, 128))]


@pytest.mark.parametrize("fname,enc", GOLDEN_MODELS)
def test_model_matches_reference_golden(cuda, golden, fname, enc):
    from light_unet.models.losses import get_loss_function
    z = golden(fname)
    model, sd = _model(z, enc, cuda)
    assert model.count_parameters()["total"] == int(z["n_params"])
    model.train()
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)
    crit = get_loss_function({"name": "FocalTverskyLoss", "alpha": 0.7, "beta": 0.3, "gamma": 0.75})
    out = model(x)
    loss = crit(out, t)
    model.zero_grad(set_to_none=True)
    loss.backward()
    torch.cuda.synchronize()
    o = out.detach().cpu().numpy()
    assert np.abs(o - z["out"]).max() <= 1e-3
    assert abs(loss.item() - float(z["loss"])) <= 1e-4 * abs(float(z["loss"]))
    grads = {k: p.grad.detach().cpu().numpy() for k, p in model.named_parameters()}
    errs, gerr = _grad_errs(grads, z)
    e32, g32 = _cpu_fp32_errs(sd, z)
    assert gerr <= max(1e-3, 2 * g32), (gerr, g32)
    bad = {k: (errs[k], e32[k]) for k in errs if errs[k] > max(1e-2, 3 * e32[k])}
    assert not bad, f"gradient errors above tolerance: {bad}"
    print(f"{fname}: out err {np.abs(o - z['out']).max():.2e}, grad L2 err {gerr:.2e} "
          f"(cpu fp32 {g32:.2e}), worst tensor {max(errs.items(), key=lambda kv: kv[1])}")


def test_dropout_masks_match_oracle(cuda, golden):
    """Dropout3d on: the kernels' channel masks, fed to the oracle, reproduce the output."""
    z = golden("model_b2_32.npz")
    model, sd = _model(z, (16, 32, 64, 128), cuda, dropout_p=0.1)
    model.train()
    x = torch.from_numpy(z["x"]).to(cuda)
    eng = model.engine
    p, sv = eng.forward(model.flat_parameters(), x, training=True, dropout_p=0.1,
                        counter=model._rng_counter)
    masks = {}
    total = dropped = 0
    for name, b in sv["blk"].items():
        k = b["recs"][1].view(x.shape[0], -1, 8)[..., 4].cpu()
        uk = np.unique(k.numpy())
        assert all(np.isclose(v, 0.0) or np.isclose(v, 1 / 0.9, rtol=1e-6) for v in uk), uk
        masks[name] = (k > 0).double()
        total += k.numel()
        dropped += int((k == 0).sum())
    assert 0 < dropped < total
    ref = U.unet_forward({k: v.double() for k, v in sd.items()}, torch.from_numpy(z["x"]).double(),
                         drop_masks=masks, drop_p=0.1)
    assert np.abs(p.cpu().numpy() - ref.numpy()).max() <= 1e-3
    # eval mode: no dropout, same as the p=0 golden
    model.eval()
    with torch.no_grad():
        pe = model(x)
    assert np.abs(pe.cpu().numpy() - z["out"]).max() <= 1e-3


def test_backward_is_deterministic(cuda, golden):
    z = golden("model_b2_32.npz")
    model, _ = _model(z, (16, 32, 64, 128), cuda)
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)
    from light_unet.models.losses import FocalTverskyLoss
    crit = FocalTverskyLoss()
    outs = []
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        loss = crit(model(x), t)
        loss.backward()
        outs.append(torch.cat([p.grad.reshape(-1) for p in model.parameters()]).cpu())
    assert torch.equal(outs[0], outs[1])


def test_trainstep_eager_graph_and_autograd_agree(cuda, golden):
    """The engine-level TrainStep (bench path), its hipGraph replay and the autograd drop-in path
    (model + criterion + torch.optim.AdamW, as trainer.py:227-232) follow the same trajectory."""
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.models.losses import FocalTverskyLoss
    from light_unet.train_step import TrainStep
    z = golden("model_b2_32.npz")
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)

    def fresh():
        m = Lightweight3DUNet(dropout_p=0.0)
        m.load_state_dict(sd)
        return m.to(cuda).train()

    steps = 4
    # (a) autograd drop-in path with torch.optim.AdamW
    m_a = fresh()
    opt = torch.optim.AdamW(m_a.parameters(), lr=1e-4, weight_decay=1e-5)
    crit = FocalTverskyLoss()
    la = []
    for _ in range(steps):
        loss = crit(m_a(x), t)
        opt.zero_grad()
        loss.backward()
        opt.step()
        la.append(loss.item())
    # (b) TrainStep eager
    m_b = fresh()
    ts = TrainStep(m_b, lr=1e-4, weight_decay=1e-5)
    lb = [ts(x, t).item() for _ in range(steps)]
    # (c) TrainStep captured in a hipGraph; capture() is side-effect free (its warm-up steps
    # run on garbage static buffers here and are rolled back), so replays start at step 1
    m_c = fresh()
    tc = TrainStep(m_c, lr=1e-4, weight_decay=1e-5)
    p0 = m_c.flat_parameters().detach().clone()
    xs, tsb = torch.full_like(x, float("nan")), torch.empty_like(t)
    tc.capture(xs, tsb, warmup=2)
    assert torch.equal(m_c.flat_parameters().detach(), p0), "capture() moved the parameters"
    assert int(m_c._rng_counter.item()) == 0 and int(tc.opt.step_t.item()) == 0
    xs.copy_(x)
    tsb.copy_(t)
    lc = []
    for _ in range(steps):
        lc.append(tc.replay().item())
    np.testing.assert_allclose(la, lb, rtol=1e-5)
    np.testing.assert_allclose(lb, lc, rtol=1e-6)
    pa = m_a.flat_parameters().detach()
    pb = m_b.flat_parameters().detach()
    pc = m_c.flat_parameters().detach()
    assert (pa - pb).abs().max().item() <= 3e-4 * steps
    assert torch.equal(pb, pc), "graph replay must be bitwise identical to eager"


def test_trainstep_fused_update_bitwise(cuda, golden, monkeypatch):
    """One process: the gradient reduction launch that also applies AdamW
    (l3u_reduce_segments_adamw) gives bitwise the parameters, moments, gradients, step and
    Dropout3d counters of the two-launch step (l3u_reduce_segments + l3u_adamw_tick)."""
    from light_unet import engine as E
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    z = golden("model_b2_32.npz")
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)
    runs = []
    for fuse in (False, True):
        monkeypatch.setattr(E, "_FUSE_ADAMW", fuse)
        m = Lightweight3DUNet(dropout_p=0.1)
        m.load_state_dict(sd)
        m = m.to(cuda).train()
        ts = TrainStep(m, lr=1e-3, weight_decay=1e-2)
        losses = [ts(x, t).item() for _ in range(3)]
        assert m.engine.applied_update == fuse
        runs.append((losses, ts.flat.clone(), ts.gflat.clone(), ts.opt.m.clone(),
                     ts.opt.v.clone(), int(ts.opt.step_t.item()), int(m._rng_counter.item()),
                     int(ts.opt.ticket.abs().sum().item())))
    a, b = runs
    assert a[0] == b[0]
    for name, u, w in zip(("params", "grads", "exp_avg", "exp_avg_sq"), a[1:5], b[1:5]):
        assert torch.equal(u, w), (name, int((u != w).sum()), float((u - w).abs().max()))
    assert a[5:] == b[5:] and b[5] == 3 and b[7] == 0


def test_state_dict_roundtrip_and_reference_keys(cuda, golden):
    z = golden("model_b1_48.npz")
    model, sd = _model(z, (16, 32, 64, 128), cuda)
    out_sd = model.state_dict()
    assert list(out_sd) == [k[2:] for k in z.files if k.startswith("w/")]
    for k, v in out_sd.items():
        assert torch.equal(v.cpu(), sd[k])
    with pytest.raises(Exception):
        model(torch.zeros(1, 1, 48, 48, 48))   # CPU input on the MI355X path fails loudly


def test_full_size_batch_independence(cuda):
    """BASELINE config 2 at full size (bs 4, 48^3): InstanceNorm and every kernel work per sample,
    so the batch-4 forward equals the four batch-1 forwards (a size-independent property at the
    benchmark shape; the fixtures cover the values at bs 1-2)."""
    from light_unet.models.unet3d import Lightweight3DUNet
    torch.manual_seed(42)
    m = Lightweight3DUNet(dropout_p=0.1).to(cuda).eval()
    rng = np.random.default_rng(49)
    x = torch.from_numpy(rng.random((4, 1, 48, 48, 48), dtype=np.float32)).to(cuda)
    with torch.no_grad():
        p4 = m(x)
        p1 = torch.cat([m(x[i:i + 1]) for i in range(4)])
    torch.cuda.synchronize()
    assert torch.isfinite(p4).all()
    assert (p4 - p1).abs().max().item() <= 1e-6


# (encoder channels, activation storage, volume edge): the fp32 16 -> 128 network, BASELINE config
# 3 (the same network with bf16 activation storage) and config 5's 32 -> 256 network (at 32^3 here:
# the protocol, not the volume, is under test; the full 64^3 step is test_fullsize_gpu's)
DP_CASES = [((16, 32, 64, 128), "f32", 32), ((16, 32, 64, 128), "bf16", 32),
            ((32, 64, 128, 256), "f32", 32)]


@pytest.mark.parametrize("enc,adt,size", DP_CASES)
def test_trainstep_data_parallel_two_ranks(cuda, tmp_path, enc, adt, size):
    """The product data-parallel step (TrainStep: 3-segment graph with eager collectives, in-kernel
    FTL gradient from all-reduced sums) on 2 ranks x bs 2 (gloo here, both ranks on this GPU;
    RCCL on a node) against the single-process bs-4 step:
      exact mode == single process on the concatenated batch (loss, flat gradient, parameters
      after an eager step and a graph replay), to fp32 summation-order rounding;
      local mode == the mean of the two half-batch single-process gradients (plain DDP);
      Dropout3d: the ranks draw different channel masks; rank 0 draws the single-process masks
      of samples 0-1 (the seed is mixed with the rank, engine.stream_seed)."""
    import os
    import socket
    import subprocess
    import sys
    from light_unet.train_step import TrainStep
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _trainstep_dist_worker as W
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(root, "tests", "_trainstep_dist_worker.py"), str(tmp_path),
           ",".join(map(str, enc)), adt, str(size)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:]
    rk = [np.load(tmp_path / f"rank{i}.npz") for i in range(2)]
    bt = W.batches(2, size)
    dtype = torch.bfloat16 if adt == "bf16" else torch.float32
    dx = [torch.from_numpy(x).to(cuda) for x, _ in bt]
    dt = [torch.from_numpy(t).to(cuda) for _, t in bt]

    def rel(a, b):
        return float(np.linalg.norm(a.astype(np.float64) - b) / np.linalg.norm(b))

    # single process, bs 4: eager step, then a second eager step
    m = W.fresh_model(cuda, 0.0, enc)
    ts = TrainStep(m, dtype=dtype)
    p0 = ts.flat.cpu().numpy().astype(np.float64)
    l1 = ts(dx[0], dt[0]).item()
    g1 = ts.gflat.cpu().numpy().astype(np.float64)
    p1 = ts.flat.cpu().numpy().astype(np.float64)
    l2 = ts(dx[1], dt[1]).item()
    p2 = ts.flat.cpu().numpy().astype(np.float64)
    for z in rk:
        assert abs(float(z["A_loss1"]) - l1) <= 1e-5 * abs(l1)
        assert abs(float(z["A_loss2"]) - l2) <= 1e-5 * abs(l2)
        assert rel(z["A_g1"], g1) <= 1e-4, rel(z["A_g1"], g1)
        # AdamW's first steps move a parameter by ~lr * g / (|g| + eps): gradients near eps
        # (1e-8) carry the fp32 summation-order differences of the two partitions (one bs-4
        # reduction vs two bs-2 reductions + all-reduce) into the update, bounded by lr per step;
        # the trajectory as a whole agrees to 1e-2 of the distance travelled
        assert np.abs(z["A_p1"] - p1).max() <= 1e-4
        assert np.abs(z["A_p2"] - p2).max() <= 2e-4
        # bf16 storage: the second step's forward re-rounds every stored activation from
        # parameters that already differ by fp32 summation order, which moves noise-level
        # gradients (e.g. the scale-invariant init_conv.shortcut.0.weight) by more than their
        # size, and AdamW turns each into an lr-sized move: measured 7.9e-2 of the distance
        # travelled (fp32 storage: < 1e-2); the first step (loss, gradient, update) is held to
        # the fp32 bounds above
        ptol = 1.5e-1 if adt == "bf16" else 1e-2
        assert np.linalg.norm(z["A_p2"] - p2) <= ptol * np.linalg.norm(p2 - p0)
    assert np.array_equal(rk[0]["A_p2"], rk[1]["A_p2"]), "ranks diverged"
    # local mode: mean of the half-batch gradients
    gh = []
    for h in range(2):
        mh = W.fresh_model(cuda, 0.0, enc)
        th = TrainStep(mh, dtype=dtype)
        th(dx[0][2 * h:2 * h + 2].contiguous(), dt[0][2 * h:2 * h + 2].contiguous())
        gh.append(th.gflat.cpu().numpy().astype(np.float64))
    gmean = 0.5 * (gh[0] + gh[1])
    for z in rk:
        assert rel(z["B_g1"], gmean) <= 1e-4, rel(z["B_g1"], gmean)
    # dropout masks: distinct per rank, rank 0 == single-process samples 0-1
    ms = W.fresh_model(cuda, 0.1, enc)
    ms.engine.set_act_dtype(dtype)
    _, sv = ms.engine.forward(ms.flat_parameters(), dx[0], training=True, dropout_p=0.1,
                              counter=ms._rng_counter, save=True)
    differ = False
    for i, pre in enumerate(ms.engine.BLOCKS):
        k0, k1 = rk[0][f"C_keep{i}"], rk[1][f"C_keep{i}"]
        differ |= not np.array_equal(k0, k1)
        ks = sv["blk"][pre]["recs"][1][:, 4].cpu().numpy()
        np.testing.assert_array_equal(k0, ks[:k0.size])
    assert differ, "both ranks drew the same Dropout3d masks"



@pytest.mark.parametrize("switch,fixture,extra", [("_RANK1", "model_b2_32.npz", {}),
                                                  ("_POOLFOLD", "model_b2_32.npz", {}),
                                                  ("_POOLFOLD", "model_b1_48.npz", {}),
                                                  ("_FRONT_R1", "model_b1_48.npz", {}),
                                                  ("_FRONT_R1", "model_b1_48.npz", {"_DWPW": False}),
                                                  ("_PAIR_BWD", "model_b1_48.npz", {}),
                                                  ("_PAIR_BWD", "model_b2_32.npz", {})])
def test_formed_on_load_gradients_bitwise(cuda, golden, switch, fixture, extra):
    """Output gradients formed on load give bitwise the gradients of the materialised tensors,
    for the FocalTversky and the given-dL/dp forms of the backward:
    _RANK1: out_conv is rank-1 (unet3d.py:201), the last block gets d(pre-sigmoid) and the
    out_conv weight (l3u_outconv_bwd_dz + the _r1 tail kernels);
    _POOLFOLD: the encoder levels' MaxPool3d backward (unet3d.py:104) inside the consuming block
    tail's loads (the _up tail kernels; at 48^3 the 48^3 and 24^3 levels);
    _FRONT_R1: the first block's rank-1 activations y1 = w1[c] * z1 and r = wsc[c] * x
    (unet3d.py:163-167, one input channel) formed on load by the fused conv2, the block tail,
    the IN-fused depthwise backward and the pointwise backwards instead of stored (48^3: the
    shapes where all of them take the rank-1 form);
    _PAIR_BWD: a block's conv2.pointwise and shortcut backwards in one launch at the 12^3 / 6^3
    levels (l3u_pw_bwd2), the shortcut writing d(input) before the depthwise backward adds to it.
    extra: engine switches held for both runs (_DWPW False: conv2 as l3u_dw3_fwd + l3u_pw_fwd, the
    rank-1 y1 formed on load by the depthwise forward).
    The output is compared too."""
    import light_unet.engine as E
    saved = {k: getattr(E, k) for k in extra}
    for k, v in extra.items():
        setattr(E, k, v)
    z = golden(fixture)
    sd = {k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")}
    x = torch.from_numpy(z["x"]).to(cuda)
    t = torch.from_numpy(z["target"]).to(cuda)
    res = []
    try:
        _formed_on_load_runs(E, switch, sd, x, t, cuda, res)
    finally:
        for k, v in saved.items():
            setattr(E, k, v)
    for name, a, b in zip(("ftl grad", "dp grad", "loss", "output"), *res):
        assert torch.equal(a, b), (name, (a - b).abs().max().item())


def _formed_on_load_runs(E, switch, sd, x, t, cuda, res):
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    for on in (True, False):
        setattr(E, switch, on)
        try:
            m = Lightweight3DUNet(dropout_p=0.1)
            m.load_state_dict(sd)
            m = m.to(cuda).train()
            ts = TrainStep(m)
            p, sv, sums = ts._fwd(x, t)
            ts._bwd(p, sv, t, sums)
            g1 = ts.gflat.clone()
            dp = torch.rand(p.shape, generator=torch.Generator().manual_seed(9)).to(cuda)
            gg = torch.zeros_like(ts.gflat)
            m.engine.backward(ts.flat, gg, sv, dp)
            torch.cuda.synchronize()
            res.append((g1, gg, ts.loss.clone(), p.clone()))
            if switch == "_FRONT_R1":
                assert (sv["blk"]["init_conv."]["y1"] is None) == on
        finally:
            setattr(E, switch, True)
