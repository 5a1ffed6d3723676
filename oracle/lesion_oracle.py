"""numpy restatement of the reference's lesion post-processing (TEST INFRASTRUCTURE — see
oracle/__init__).  Checker for light_unet/lesion.py (HIP kernels csrc/lesion.hip).

Follows:
  get_connected_components   light_unet/models/metrics.py:38-63 — scipy.ndimage.label with its
                             default structure for the array's rank (face neighbours: 6 for a
                             [D, H, W] volume, 8 for a batched [B, D, H, W] array), components
                             numbered in the order of their first voxel in a C-order scan;
                             min_size drops smaller components and relabels (:52-61)
  match_components           metrics.py:127-213 (IoU matrix in float32, centres of mass in mm --
                             the three LEADING coordinates of the array, :99-124 -- greedy
                             matching in predicted-component order)
  calculate_lesion_metrics   metrics.py:216-287
  bounding boxes             light_unet/core/inferencer.py:62-111
The labelling is restated as min-label propagation over the face neighbours with pointer jumping
(every foreground voxel ends holding the smallest linear index of its component), then ranked —
not scipy's two-pass algorithm, but the same partition and numbering.  Pinned by
tests/golden/lesion.npz (made by running the reference's metrics.py, scipy 1.15.3).
"""
import numpy as np


def label6(mask):
    """(labels int32, n): face-connected components of mask != 0 (any rank), numbered by first
    voxel."""
    m = np.asarray(mask) != 0
    n_vox = m.size
    idx = np.arange(n_vox, dtype=np.int64).reshape(m.shape)
    lab = np.where(m, idx, n_vox)                      # background: a sentinel above every index
    while True:
        new = lab.copy()
        for ax in range(m.ndim):
            for sh in (1, -1):
                nb = np.roll(lab, sh, axis=ax)
                valid = np.roll(m, sh, axis=ax)
                # np.roll wraps around: the wrapped slab is not a neighbour
                sl = [slice(None)] * m.ndim
                sl[ax] = slice(0, 1) if sh == 1 else slice(-1, None)
                valid[tuple(sl)] = False
                new = np.where(m & valid, np.minimum(new, nb), new)
        flat = new.reshape(-1)
        fg = flat < n_vox
        flat[fg] = flat[flat[fg]]                      # pointer jump: lab <- lab[lab]
        new = flat.reshape(m.shape)
        if np.array_equal(new, lab):
            break
        lab = new
    roots = np.unique(lab[m])
    out = np.zeros(m.shape, np.int32)
    out[m] = np.searchsorted(roots, lab[m]).astype(np.int32) + 1
    return out, int(roots.size)


def get_connected_components(mask, min_size=0):
    lab, n = label6(mask)
    if min_size > 0:
        sizes = np.bincount(lab.ravel(), minlength=n + 1)
        small = sizes < min_size
        small[0] = False
        lab = lab.copy()
        lab[small[lab]] = 0
        lab, n = label6(lab > 0)
    return lab, n


def centers(lab, n):
    """Per-component centres of mass over the array's three leading coordinates."""
    if n == 0:
        return np.empty((0, 3), np.float64)
    coords = np.indices(lab.shape).reshape(lab.ndim, -1).astype(np.float64)
    cnt = np.bincount(lab.ravel(), minlength=n + 1)[1:].astype(np.float64)
    return np.stack([np.bincount(lab.ravel(), weights=coords[d], minlength=n + 1)[1:] / cnt
                     for d in range(3)], axis=1)


def match_components(pl, tl, iou_threshold=0.1, distance_threshold_mm=10.0, spacing=(4.0, 4.0, 4.0)):
    npred, ntgt = int(pl.max()), int(tl.max())
    if npred == 0 or ntgt == 0:
        return [], list(range(1, npred + 1)), list(range(1, ntgt + 1))
    pf, tf = pl.ravel().astype(np.int64), tl.ravel().astype(np.int64)
    inter = np.bincount(pf * (ntgt + 1) + tf, minlength=(npred + 1) * (ntgt + 1)).reshape(npred + 1, ntgt + 1)
    inter[0, :] = 0
    inter[:, 0] = 0
    ps, ts = np.bincount(pf, minlength=npred + 1), np.bincount(tf, minlength=ntgt + 1)
    union = ps[:, None] + ts[None, :] - inter
    iou = np.divide(inter, union, out=np.zeros_like(inter, dtype=np.float32), where=union > 0)
    sp = np.asarray(spacing, np.float64)
    dist = np.linalg.norm((centers(pl, npred) * sp)[:, None, :] - (centers(tl, ntgt) * sp)[None, :, :], axis=2)
    matches, taken = [], np.zeros(ntgt, bool)
    for p in range(1, npred + 1):
        ok = ~taken & ((iou[p, 1:] >= iou_threshold) | (dist[p - 1] <= distance_threshold_mm))
        if ok.any():
            b = int(np.argmax(np.where(ok, iou[p, 1:], -np.inf)))
            matches.append((p, b + 1))
            taken[b] = True
    mp = {p for p, _ in matches}
    return matches, [i for i in range(1, npred + 1) if i not in mp], [i for i in range(1, ntgt + 1) if not taken[i - 1]]


def squeeze(a):
    """metrics.py:236-244: [B, 1, D, H, W] -> [B, D, H, W]; [1, D, H, W] -> [D, H, W]."""
    a = np.asarray(a)
    if a.ndim == 5:
        a = a[:, 0]
    if a.ndim == 4 and a.shape[0] == 1:
        a = a[0]
    return a


def lesion_metrics(pred, target, threshold=0.5, min_size_voxels=0, iou_threshold=0.1,
                   distance_threshold_mm=10.0, spacing=(4.0, 4.0, 4.0)):
    pred, target = squeeze(pred), squeeze(target)
    pl, npred = get_connected_components(np.asarray(pred) >= threshold, min_size_voxels)
    tl, ntgt = get_connected_components(np.asarray(target) >= 0.5, min_size_voxels)
    if ntgt == 0:
        if npred == 0:
            return {"recall": 1.0, "precision": 1.0, "f1": 1.0, "tp": 0, "fp": 0, "fn": 0}
        return {"recall": 0.0, "precision": 0.0, "f1": 0.0, "tp": 0, "fp": npred, "fn": 0}
    if npred == 0:
        return {"recall": 0.0, "precision": 0.0, "f1": 0.0, "tp": 0, "fp": 0, "fn": ntgt}
    m, up, ut = match_components(pl, tl, iou_threshold, distance_threshold_mm, spacing)
    tp, fp, fn = len(m), len(up), len(ut)
    r = tp / (tp + fn) if tp + fn else 0.0
    p = tp / (tp + fp) if tp + fp else 0.0
    return {"recall": r, "precision": p, "f1": 2 * p * r / (p + r) if p + r else 0.0,
            "tp": tp, "fp": fp, "fn": fn}


def bboxes(prob, threshold=0.3, min_volume_cc=0.5, spacing=(4.0, 4.0, 4.0), expansion_voxels=0):
    vcc = spacing[0] * spacing[1] * spacing[2] / 1000.0
    lab, n = get_connected_components(prob >= threshold, int(np.ceil(min_volume_cc / vcc)))
    out = []
    for c in range(1, n + 1):
        cm = lab == c
        co = np.argwhere(cm)
        lo = np.maximum(0, co.min(0) - expansion_voxels)
        hi = np.minimum(np.array(prob.shape) - 1, co.max(0) + expansion_voxels)
        out.append({"mask_id": c, "bbox_voxel": [int(lo[0]), int(hi[0]), int(lo[1]), int(hi[1]),
                                                 int(lo[2]), int(hi[2])],
                    "volume_cc": float(cm.sum() * vcc), "confidence": float(prob[cm].max())})
    return out
