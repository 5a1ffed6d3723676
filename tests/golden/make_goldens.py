"""Generate the golden fixtures under tests/golden/ from the REFERENCE implementation.

Run here (the survey container, where /root/reference exists) with
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py
It imports the reference modules BY FILE PATH (the package import needs nibabel):
  - /root/reference/light_unet/models/unet3d.py   (Lightweight3DUNet, ResidualBlock, DownBlock, UpBlock)
  - /root/reference/light_unet/models/losses.py   (FocalTverskyLoss, get_loss_function)
  - /root/reference/light_unet/utils.py           (sliding_window_inference_3d, _get_gaussian_importance_map)
and writes inputs + expected outputs as .npz DATA (no reference source is copied).
Nothing under tests/ or the GPU box ever imports the reference; only this generator does.

All seeds are recorded in each fixture (`seed` arrays).  The whole-model goldens run the
reference in float64 so they are an accuracy anchor for both the oracle and the HIP path.
"""
import importlib.util
import os
import sys

sys.dont_write_bytecode = True

import numpy as np
import torch

REF = os.environ.get("L3U_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


unet3d = _load("ref_unet3d", "light_unet/models/unet3d.py")
losses = _load("ref_losses", "light_unet/models/losses.py")
rutils = _load("ref_utils", "light_unet/utils.py")


def perturb_affine(model, seed):
    """InstanceNorm affine params init to (1, 0) and convT bias is tiny; perturb them so the
    fixtures exercise gamma/beta (seeded, recorded)."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, p in model.named_parameters():
            leaf = name.split(".")
            is_norm = any(s.startswith("norm") for s in leaf) or (".shortcut.1." in name)
            if is_norm and name.endswith("weight"):
                p.add_(0.1 * torch.randn(p.shape, generator=g, dtype=p.dtype))
            elif is_norm and name.endswith("bias"):
                p.copy_(0.1 * torch.randn(p.shape, generator=g, dtype=p.dtype))


def sd_to_np(model):
    return {("w/" + k): v.detach().cpu().numpy().astype(np.float32) for k, v in model.state_dict().items()}


def grads_to_np(model):
    return {("g/" + k): p.grad.detach().cpu().numpy().astype(np.float32)
            for k, p in model.named_parameters()}


def model_golden(fname, enc, shape, seed, fp64=True, full=True, **variant):
    """Whole Lightweight3DUNet forward + FocalTversky + backward (dropout_p=0: Dropout3d RNG
    cannot be bit-matched).  Inputs: x ~ U[0,1), target = U[0,1) > 0.97.
    variant: use_depthwise_separable / use_grouped / groups constructor keywords."""
    torch.manual_seed(42)                                  # trainer.py:44 seed
    model = unet3d.Lightweight3DUNet(encoder_channels=list(enc), dropout_p=0.0, **variant)
    perturb_affine(model, seed + 1000)
    weights = sd_to_np(model)
    rng = np.random.default_rng(seed)
    x = rng.random(shape, dtype=np.float32)
    t = (rng.random(shape) > 0.97).astype(np.float32)
    dt = torch.float64 if fp64 else torch.float32
    model = model.to(dt)
    model.train()                                         # IN uses instance stats either way
    xt = torch.from_numpy(x).to(dt)
    tt = torch.from_numpy(t).to(dt)
    out = model(xt)
    crit = losses.get_loss_function({"name": "FocalTverskyLoss", "alpha": 0.7, "beta": 0.3, "gamma": 0.75})
    loss = crit(out, tt)
    loss.backward()
    rec = dict(weights)
    rec.update(x=x, target=t, loss=np.array(loss.item()), seed=np.array(seed),
               enc=np.array(enc), n_params=np.array(model.count_parameters()["total"]))
    for k, v in variant.items():
        rec["variant/" + k] = np.array(v)
    o = out.detach().numpy().astype(np.float32)
    if full:
        rec["out"] = o
        rec.update(grads_to_np(model))
    else:
        # large config: checksum + sampled voxels + per-tensor grad norms + a few grad entries
        flat = o.reshape(-1)
        idx = np.random.default_rng(seed + 7).choice(flat.size, 4096, replace=False)
        rec.update(out_idx=idx.astype(np.int64), out_sample=flat[idx], out_sum=np.array(o.astype(np.float64).sum()),
                   out_sumsq=np.array((o.astype(np.float64) ** 2).sum()))
        for k, p in model.named_parameters():
            gg = p.grad.detach().numpy()
            rec["gnorm/" + k] = np.array(np.linalg.norm(gg.reshape(-1)))
            rec["gmaxabs/" + k] = np.array(np.abs(gg).max())
    np.savez_compressed(os.path.join(OUT, fname), **rec)
    print(fname, "loss", loss.item(), "params", rec["n_params"])


BLOCK_CASES = [
    ("rb_a", lambda: unet3d.ResidualBlock(3, 8, dropout_p=0.0), [(2, 3, 7, 6, 9)]),
    ("rb_id", lambda: unet3d.ResidualBlock(8, 8, dropout_p=0.0), [(2, 8, 5, 7, 6)]),
    ("rb_c1", lambda: unet3d.ResidualBlock(1, 4, use_grouped=False, dropout_p=0.0), [(1, 1, 9, 8, 10)]),
    ("down", lambda: unet3d.DownBlock(4, 8, dropout_p=0.0), [(2, 4, 10, 8, 12)]),
    ("up", lambda: unet3d.UpBlock(8, 4, dropout_p=0.0), [(2, 8, 3, 4, 5), (2, 4, 6, 8, 10)]),
]
# use_depthwise_separable=False: GroupedConv3d (unet3d.py:26-34) and dense nn.Conv3d (:49, :60)
BLOCK_CASES_G = [
    ("g_rb", lambda: unet3d.ResidualBlock(8, 16, use_depthwise_separable=False, dropout_p=0.0),
     [(2, 8, 6, 7, 5)]),
    ("g_rb_id", lambda: unet3d.ResidualBlock(16, 16, use_depthwise_separable=False, groups=4,
                                             dropout_p=0.0), [(2, 16, 5, 6, 7)]),
    ("g_rb_mixed", lambda: unet3d.ResidualBlock(4, 8, use_depthwise_separable=False, groups=8,
                                                dropout_p=0.0), [(1, 4, 6, 5, 8)]),
    ("d_rb", lambda: unet3d.ResidualBlock(3, 6, use_depthwise_separable=False, use_grouped=False,
                                          dropout_p=0.0), [(2, 3, 5, 6, 7)]),
    ("g_up", lambda: unet3d.UpBlock(16, 8, use_depthwise_separable=False, dropout_p=0.0),
     [(2, 16, 3, 4, 2), (2, 8, 6, 8, 4)]),
]


def block_goldens(cases=None, fname="blocks.npz"):
    """Per-block KATs at small ragged shapes: ResidualBlock (Cin!=Cout and identity shortcut),
    DownBlock, UpBlock (unet3d.py:37-143), fp64, dropout 0, with a random upstream gradient."""
    rec = {}
    cases = BLOCK_CASES if cases is None else cases
    for i, (name, ctor, shapes) in enumerate(cases):
        torch.manual_seed(100 + i)
        blk = ctor()
        perturb_affine(blk, 200 + i)
        blk = blk.to(torch.float64)
        rng = np.random.default_rng(300 + i)
        ins = [rng.standard_normal(s) for s in shapes]
        ts = [torch.from_numpy(a).requires_grad_(True) for a in ins]
        out = blk(*ts)
        dy = rng.standard_normal(tuple(out.shape))
        out.backward(torch.from_numpy(dy))
        rec[f"{name}/dy"] = dy.astype(np.float32)
        rec[f"{name}/out"] = out.detach().numpy().astype(np.float32)
        for j, (a, tt) in enumerate(zip(ins, ts)):
            rec[f"{name}/in{j}"] = a.astype(np.float32)
            rec[f"{name}/din{j}"] = tt.grad.numpy().astype(np.float32)
        for k, v in blk.state_dict().items():
            rec[f"{name}/w/{k}"] = v.numpy().astype(np.float32)
        for k, p in blk.named_parameters():
            rec[f"{name}/g/{k}"] = p.grad.numpy().astype(np.float32)
    # inputs were generated in fp64 then rounded to fp32 for storage; regenerate the outputs from the
    # rounded inputs so consumers see a self-consistent pair
    for i, (name, ctor, shapes) in enumerate(cases):
        torch.manual_seed(100 + i)
        blk = ctor()
        blk.load_state_dict({k[len(name) + 3:]: torch.from_numpy(v) for k, v in rec.items()
                             if k.startswith(name + "/w/")})
        blk = blk.to(torch.float64)
        ts = [torch.from_numpy(rec[f"{name}/in{j}"].astype(np.float64)).requires_grad_(True)
              for j in range(len(shapes))]
        out = blk(*ts)
        out.backward(torch.from_numpy(rec[f"{name}/dy"].astype(np.float64)))
        rec[f"{name}/out"] = out.detach().numpy().astype(np.float32)
        for j, tt in enumerate(ts):
            rec[f"{name}/din{j}"] = tt.grad.numpy().astype(np.float32)
        for k, p in blk.named_parameters():
            rec[f"{name}/g/{k}"] = p.grad.numpy().astype(np.float32)
    np.savez_compressed(os.path.join(OUT, fname), **rec)
    print(fname, len(rec), "arrays")


def ftl_goldens():
    """FocalTverskyLoss (losses.py:11-54) forward + d/dpred in fp64, incl. edge cases:
    empty-lesion target, all-ones target, saturated predictions, non-default alpha/beta/gamma."""
    rec = {}
    rng = np.random.default_rng(7)
    cases = {
        "rand": (rng.random((2, 1, 8, 9, 10)), (rng.random((2, 1, 8, 9, 10)) > 0.9), (0.7, 0.3, 0.75)),
        "empty": (rng.random((1, 1, 6, 6, 6)), np.zeros((1, 1, 6, 6, 6), bool), (0.7, 0.3, 0.75)),
        "full": (rng.random((1, 1, 6, 6, 6)), np.ones((1, 1, 6, 6, 6), bool), (0.7, 0.3, 0.75)),
        "sat": (np.clip(rng.random((2, 1, 5, 5, 5)) * 3 - 1, 0, 1), (rng.random((2, 1, 5, 5, 5)) > 0.5),
                (0.7, 0.3, 0.75)),
        "params": (rng.random((3, 1, 7, 5, 6)), (rng.random((3, 1, 7, 5, 6)) > 0.8), (0.5, 0.5, 1.5)),
    }
    for name, (p, t, (a, b, g)) in cases.items():
        p32 = p.astype(np.float32)
        t32 = t.astype(np.float32)
        pt = torch.from_numpy(p32.astype(np.float64)).requires_grad_(True)
        crit = losses.FocalTverskyLoss(alpha=a, beta=b, gamma=g)
        loss = crit(pt, torch.from_numpy(t32.astype(np.float64)))
        loss.backward()
        rec[f"{name}/pred"] = p32
        rec[f"{name}/target"] = t32
        rec[f"{name}/abg"] = np.array([a, b, g])
        rec[f"{name}/loss"] = np.array(loss.item())
        rec[f"{name}/dpred"] = pt.grad.numpy()
    # error behaviour: alpha + beta != 1 asserts (losses.py:28); unknown name raises (losses.py:147)
    try:
        losses.FocalTverskyLoss(alpha=0.6, beta=0.3)
        rec["err/assert_ab"] = np.array(0)
    except AssertionError:
        rec["err/assert_ab"] = np.array(1)
    try:
        losses.get_loss_function({"name": "Nope"})
        rec["err/unknown"] = np.array(0)
    except ValueError:
        rec["err/unknown"] = np.array(1)
    np.savez_compressed(os.path.join(OUT, "ftl.npz"), **rec)
    print("ftl.npz", len(rec))


def sliding_goldens():
    """sliding_window_inference_3d (utils.py:11-139) with the bs=1 48^3 golden weights (fp32 CPU,
    exactly as the reference runs it), on ragged volumes incl. one smaller than the patch."""
    torch.manual_seed(42)
    model = unet3d.Lightweight3DUNet(dropout_p=0.1)
    perturb_affine(model, 11)
    rec = sd_to_np(model)
    imp = rutils._get_gaussian_importance_map((48, 48, 48))
    rec["importance_48"] = imp
    rng = np.random.default_rng(5)
    for name, shape in {"v64_56_72": (64, 56, 72), "v40_52_48": (40, 52, 48)}.items():
        vol = rng.random(shape, dtype=np.float32) * 0.3
        prob = rutils.sliding_window_inference_3d(vol, model, (48, 48, 48), 0.5, torch.device("cpu"), True)
        rec[f"{name}/image"] = vol
        rec[f"{name}/prob"] = prob.astype(np.float32)
        for thr in (0.1, 0.3, 0.5, 0.7):
            rec[f"{name}/mask_{thr}"] = (prob >= thr)
            # margin: distance of the closest voxel to the threshold (tests skip bit-exactness if tiny)
            rec[f"{name}/margin_{thr}"] = np.array(np.abs(prob - thr).min())
    np.savez_compressed(os.path.join(OUT, "sliding.npz"), **rec)
    print("sliding.npz", len(rec))


def variant_goldens():
    """The use_depthwise_separable=False network family (grouped and dense 3^3 convs)."""
    block_goldens(BLOCK_CASES_G, "blocks_g.npz")
    model_golden("model_g_b2_16.npz", (8, 16, 32, 64), (2, 1, 16, 16, 16), seed=45,
                 use_depthwise_separable=False, use_grouped=True, groups=8)
    model_golden("model_d_b1_16.npz", (4, 8, 16, 32), (1, 1, 16, 16, 16), seed=46,
                 use_depthwise_separable=False, use_grouped=False, groups=8)


def _blobs(rng, shape, n, rmax, centers=None):
    """A smooth synthetic probability map: n Gaussian blobs on a low background (at `centers`
    when given, else uniform)."""
    zz, yy, xx = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
    p = rng.random(shape) * 0.05
    for i in range(n):
        c = centers[i] if centers is not None else [rng.uniform(0, s) for s in shape]
        r = rng.uniform(1.0, rmax)
        amp = rng.uniform(0.3, 1.0)
        p = np.maximum(p, amp * np.exp(-((zz - c[0]) ** 2 + (yy - c[1]) ** 2 + (xx - c[2]) ** 2) / (2 * r * r)))
    return p.astype(np.float32)


def lesion_goldens():
    """Lesion post-processing from the REFERENCE light_unet/models/metrics.py:
    get_connected_components (ndimage.label; min_size filter), match_components,
    calculate_lesion_metrics, calculate_metrics.  The bounding boxes of inferencer.py:62-111 are
    restated here on the reference's own labels (that module imports nibabel, absent here)."""
    metrics = _load("ref_metrics", "light_unet/models/metrics.py")
    rng = np.random.default_rng(49)
    rec = {}
    masks = {
        "rand30": rng.random((20, 24, 28)) < 0.30,
        "rand50": rng.random((17, 19, 23)) < 0.50,            # near percolation: long snakes
        "sparse": rng.random((16, 16, 16)) < 0.05,
        "empty": np.zeros((8, 9, 10), bool),
        "full": np.ones((8, 9, 10), bool),
        "single": np.zeros((9, 9, 9), bool),
        "checker": (np.indices((10, 12, 14)).sum(0) % 2) == 0,  # no face neighbours at all
    }
    masks["single"][4, 5, 6] = True
    for name, m in masks.items():
        lab, num = metrics.get_connected_components(m.astype(np.int32))
        rec[f"cc/{name}/mask"] = m
        rec[f"cc/{name}/labels"] = lab.astype(np.int32)
        rec[f"cc/{name}/num"] = np.array(num)
        lab5, num5 = metrics.get_connected_components(m.astype(np.int32), min_size=5)
        rec[f"cc/{name}/labels_min5"] = lab5.astype(np.int32)
        rec[f"cc/{name}/num_min5"] = np.array(num5)
    # lesion matching / metrics on synthetic probability maps and targets
    cases = []
    for i, (shape, npred, ntgt) in enumerate([((32, 36, 40), 9, 7), ((24, 28, 20), 4, 0),
                                              ((28, 28, 28), 0, 5), ((30, 26, 34), 12, 10)]):
        # targets at random centres; predictions hit most of them (jittered 0-3 voxels, so both
        # IoU and centre-distance matches occur) plus false positives elsewhere
        tc = [[rng.uniform(0, s) for s in shape] for _ in range(ntgt)]
        hit = [[c + rng.uniform(-3, 3) for c in cc] for cc in tc[: max(0, ntgt - 2)]]
        pc = (hit + [[rng.uniform(0, s) for s in shape] for _ in range(npred)])[:npred]
        pred = _blobs(rng, shape, len(pc), 3.5, pc) if npred else (rng.random(shape) * 0.05).astype(np.float32)
        tgt = (_blobs(rng, shape, ntgt, 3.0, tc) >= 0.5).astype(np.float32) if ntgt else np.zeros(shape, np.float32)
        cases.append((pred, tgt))
        rec[f"lm/{i}/pred"] = pred
        rec[f"lm/{i}/target"] = tgt
        for thr in (0.3, 0.5):
            m = metrics.calculate_lesion_metrics(pred, tgt, threshold=thr, spacing=(4.0, 4.0, 4.0))
            for k, v in m.items():
                rec[f"lm/{i}/thr{thr}/{k}"] = np.array(v)
        m2 = metrics.calculate_lesion_metrics(pred, tgt, threshold=0.3, min_size_voxels=6,
                                              iou_threshold=0.2, distance_threshold_mm=6.0,
                                              spacing=(2.0, 3.0, 4.0))
        for k, v in m2.items():
            rec[f"lm/{i}/opts/{k}"] = np.array(v)
        pl, _ = metrics.get_connected_components((pred >= 0.3).astype(np.int32))
        tl, _ = metrics.get_connected_components((tgt >= 0.5).astype(np.int32))
        mt, up, ut = metrics.match_components(pl, tl, 0.1, 10.0, (4.0, 4.0, 4.0))
        rec[f"lm/{i}/matches"] = np.array(mt, dtype=np.int64).reshape(-1, 2)
        rec[f"lm/{i}/unmatched_pred"] = np.array(up, dtype=np.int64)
        rec[f"lm/{i}/unmatched_target"] = np.array(ut, dtype=np.int64)
    agg = metrics.calculate_metrics([c[0] for c in cases], [c[1] for c in cases], threshold=0.3,
                                    spacing=[(4.0, 4.0, 4.0), (2.0, 2.0, 2.0), (4.0, 4.0, 4.0), (3.0, 4.0, 5.0)])
    for k, v in agg.items():
        rec[f"agg/{k}"] = np.array(v)
    # bounding boxes (inferencer.py:62-111 restated on the reference's labels)
    prob = _blobs(rng, (40, 44, 36), 10, 4.0)
    spacing, expand = (4.0, 4.0, 4.0), 2
    vcc = spacing[0] * spacing[1] * spacing[2] / 1000.0
    minv = int(np.ceil(0.5 / vcc))
    lab, num = metrics.get_connected_components((prob >= 0.3).astype(np.int32), min_size=minv)
    boxes = []
    for cid in range(1, num + 1):
        cm = lab == cid
        co = np.argwhere(cm)
        lo, hi = co.min(0), co.max(0)
        lo = np.maximum(0, lo - expand)
        hi = np.minimum(np.array(prob.shape) - 1, hi + expand)
        boxes.append([cid, lo[0], hi[0], lo[1], hi[1], lo[2], hi[2]])
        rec[f"bb/{cid}/volume_cc"] = np.array(cm.sum() * vcc)
        rec[f"bb/{cid}/confidence"] = np.array(prob[cm].max())
    rec["bb/prob"] = prob
    rec["bb/boxes"] = np.array(boxes, dtype=np.int64).reshape(-1, 7)
    # batched [B, D, H, W] arrays: ndimage.label labels them as ONE 4-dimensional array (the batch
    # axis is a fourth face neighbour) and the centres keep the leading coordinates (b, z, y)
    rb = np.random.default_rng(50)
    m4 = rb.random((2, 12, 14, 16)) < 0.3
    m4[1] |= m4[0] & (rb.random((12, 14, 16)) < 0.5)   # shared voxels join items across the batch
    lab4, num4 = metrics.get_connected_components(m4.astype(np.int32))
    rec["b4/cc/mask"] = m4
    rec["b4/cc/labels"] = lab4.astype(np.int32)
    rec["b4/cc/num"] = np.array(num4)
    lab4m, num4m = metrics.get_connected_components(m4.astype(np.int32), min_size=5)
    rec["b4/cc/labels_min5"] = lab4m.astype(np.int32)
    rec["b4/cc/num_min5"] = np.array(num4m)
    shape = (24, 20, 28)
    preds, tgts = [], []
    for k in range(2):
        tcen = [[rb.uniform(0, s) for s in shape] for _ in range(6)]
        hit = [[c + rb.uniform(-3, 3) for c in cc] for cc in tcen[:4]]
        pcen = hit + [[rb.uniform(0, s) for s in shape] for _ in range(4)]
        preds.append(_blobs(rb, shape, len(pcen), 3.5, pcen))
        tgts.append((_blobs(rb, shape, len(tcen), 3.0, tcen) >= 0.5).astype(np.float32))
    pred4, tgt4 = np.stack(preds)[:, None], np.stack(tgts)[:, None]   # [2, 1, D, H, W]
    rec["b4/lm/pred"], rec["b4/lm/target"] = pred4, tgt4
    for thr in (0.3, 0.5):
        m = metrics.calculate_lesion_metrics(pred4, tgt4, threshold=thr, spacing=(4.0, 4.0, 4.0))
        for k, v in m.items():
            rec[f"b4/lm/thr{thr}/{k}"] = np.array(v)
    m2 = metrics.calculate_lesion_metrics(pred4[:, 0], tgt4[:, 0], threshold=0.3, min_size_voxels=4,
                                          iou_threshold=0.2, distance_threshold_mm=6.0,
                                          spacing=(2.0, 3.0, 4.0))
    for k, v in m2.items():
        rec[f"b4/lm/opts/{k}"] = np.array(v)
    pl4, _ = metrics.get_connected_components((pred4[:, 0] >= 0.3).astype(np.int32))
    tl4, _ = metrics.get_connected_components((tgt4[:, 0] >= 0.5).astype(np.int32))
    for nm, (a, b) in (("b2", (pl4, tl4)), ("b1", (pl4[:1], tl4[:1]))):   # b1: [1, D, H, W] arrays
        mt, up, ut = metrics.match_components(a, b, 0.1, 10.0, (4.0, 4.0, 4.0))
        rec[f"b4/match/{nm}/matches"] = np.array(mt, dtype=np.int64).reshape(-1, 2)
        rec[f"b4/match/{nm}/unmatched_pred"] = np.array(up, dtype=np.int64)
        rec[f"b4/match/{nm}/unmatched_target"] = np.array(ut, dtype=np.int64)
    agg = metrics.calculate_metrics(pred4, tgt4, threshold=0.3)   # [B, 1, D, H, W]: one case per item
    for k, v in agg.items():
        rec[f"b4/agg/{k}"] = np.array(v)
    np.savez_compressed(os.path.join(OUT, "lesion.npz"), **rec)
    print("lesion.npz", len(rec), "arrays")


def ragged_goldens():
    """Volumes the MI355X path once refused: D/H/W not divisible by 8 (the UpBlock pad branch,
    unet3d.py:130-138, fires at every decoder level) and planes above 64x64 (80x80)."""
    model_golden("model_b1_40_44_36.npz", (16, 32, 64, 128), (1, 1, 40, 44, 36), seed=47)
    model_golden("model_b1_24_80_80.npz", (16, 32, 64, 128), (1, 1, 24, 80, 80), seed=48)


if __name__ == "__main__":
    torch.set_num_threads(8)
    if sys.argv[1:] == ["variants"]:
        variant_goldens()
        sys.exit(0)
    if sys.argv[1:] == ["lesion"]:
        lesion_goldens()
        sys.exit(0)
    if sys.argv[1:] == ["ragged"]:
        ragged_goldens()
        sys.exit(0)
    if sys.argv[1:] == ["c32"]:
        model_golden("model_c32_b1_64.npz", (32, 64, 128, 256), (1, 1, 64, 64, 64), seed=44)
        sys.exit(0)
    variant_goldens()
    block_goldens()
    ftl_goldens()
    model_golden("model_b2_32.npz", (16, 32, 64, 128), (2, 1, 32, 32, 32), seed=42)
    model_golden("model_b1_48.npz", (16, 32, 64, 128), (1, 1, 48, 48, 48), seed=43)
    model_golden("model_c32_b1_64.npz", (32, 64, 128, 256), (1, 1, 64, 64, 64), seed=44)
    ragged_goldens()
    lesion_goldens()
    sliding_goldens()
