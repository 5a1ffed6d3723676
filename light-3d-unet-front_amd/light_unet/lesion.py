"""Lesion post-processing on the MI355X: connected components, lesion matching, lesion metrics and
bounding boxes, mirroring the reference's host functions

    get_connected_components   light_unet/models/metrics.py:38-63
    match_components           light_unet/models/metrics.py:127-213
    calculate_lesion_metrics   light_unet/models/metrics.py:216-287
    calculate_metrics          light_unet/models/metrics.py:306-404
    extract_bboxes             light_unet/core/inferencer.py:62-111

with the same signatures, return types and numbering.  The per-voxel work runs in the HIP
kernels of csrc/lesion.hip (include/l3u.h, l3u_ccl_*): labelling (scipy.ndimage.label's
6-connectivity and first-encounter numbering), per-component sizes / coordinate sums / bounding
boxes / peak probability (exact integer atomics), and the pairwise overlap counts of two
labellings.  What stays on the host is O(components): the greedy matching loop and the final
ratios, written as the reference writes them so the floats agree bit for bit.  Inputs may be
numpy arrays (uploaded once) or device tensors; there is no CPU fallback.
"""
import math

import numpy as np
import torch

from . import _native as nat

# stats columns (csrc/lesion.hip)
_SIZE, _SUM, _MIN, _MAX, _PMAX = 0, slice(1, 4), slice(4, 7), slice(7, 10), 10


def _device():
    if not torch.cuda.is_available():
        raise nat.NativeError("lesion post-processing runs on the ROCm device; no GPU is visible "
                              "(there is no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


def _dims(shape):
    """(B, D, H, W, lead4) of a labelled / thresholded array, in ndimage.label's own terms: a
    [D, H, W] volume (B = 1, coordinates z, y, x) or a [B, D, H, W] array labelled as ONE
    4-dimensional array (the batch axis is a fourth face neighbour; the reference's centres keep
    the leading coordinates b, z, y, metrics.py:99-124).  Other ranks are not taken."""
    shape = tuple(int(v) for v in shape)
    if len(shape) == 3:
        return (1,) + shape + (0,)
    if len(shape) == 4:
        return shape + (1,)
    raise ValueError(f"expected a [D, H, W] volume or a [B, D, H, W] array, got shape {shape}")


def _volume(a, dev, keep_f64=False):
    """The array (3- or 4-dimensional, shape kept) as float32 on the device.  keep_f64: a float64
    input stays float64 (the reference thresholds float64 maps in float64)."""
    t = a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(np.asarray(a)))
    _dims(t.shape)
    if t.dtype == torch.bool:
        t = t.to(torch.uint8)
    dt = torch.float64 if (keep_f64 and t.dtype == torch.float64) else torch.float32
    return t.to(device=dev, dtype=dt).contiguous()


def _foreground(vol, threshold, dev):
    """(volume, threshold) for l3u_ccl_label, which compares in float32.  A float64 map is
    compared in float64 on the device first (`vol >= threshold` as metrics.py:245 /
    inferencer.py:64 evaluate it in numpy), so values between float32(threshold) and threshold
    classify as the reference classifies them; the kernel then labels the 0/1 mask."""
    v = _volume(vol, dev, keep_f64=True)
    if v.dtype == torch.float64:
        return (v >= float(threshold)).to(torch.float32), 0.5
    return v, threshold


class Components:
    """A labelling on the device: `labels` int32 (the input's [D, H, W] or [B, D, H, W] shape),
    `num` components, `stats` uint64 [num, 12] (host) as l3u_ccl_stats_b writes them."""

    def __init__(self, labels, num, stats):
        self.labels, self.num, self.stats = labels, int(num), stats
        self.pmax64 = None   # float64 per-component maxima of a float64 prob map (label(prob=))

    def sizes(self):
        return self.stats[:, _SIZE].astype(np.int64)

    def centers(self):
        """Centres of mass in voxels, scipy.ndimage.center_of_mass's float64 sum / count (the
        three leading coordinates of the array, as metrics.py:99-124 keeps them)."""
        if self.num == 0:
            return np.empty((0, 3), dtype=np.float64)
        return self.stats[:, _SUM].astype(np.float64) / self.stats[:, _SIZE:_SIZE + 1].astype(np.float64)

    def numpy(self):
        return self.labels.cpu().numpy()


def label(vol, threshold=0.5, min_size=0, prob=None):
    """Components of (vol >= threshold); min_size > 0 drops smaller ones and renumbers the rest in
    order (metrics.py:52-61: removing whole components never changes the others' connectivity, so
    ndimage.label of the survivors is the order-preserving rank).  prob: optional volume whose
    per-component maximum lands in stats[:, 10] (float32 bits)."""
    dev = _device()
    v, threshold = _foreground(vol, threshold, dev)
    B, D, H, W, lead4 = _dims(v.shape)
    n = v.numel()
    st = nat.stream()
    parent = torch.empty(n, dtype=torch.int32, device=dev)
    lab = torch.empty(v.shape, dtype=torch.int32, device=dev)
    nch = nat.query("l3u_ccl_nchunks", n)
    cnt = torch.empty(nch + 1, dtype=torch.int32, device=dev)
    nat.call("l3u_ccl_label_b", v.data_ptr(), float(threshold), parent.data_ptr(), lab.data_ptr(),
             cnt.data_ptr(), B, D, H, W, st)
    num = int(cnt[nch].item())
    if num == 0:
        return Components(lab, 0, np.zeros((0, 12), dtype=np.uint64))
    pv = _volume(prob, dev, keep_f64=True) if prob is not None else None
    if pv is not None and tuple(pv.shape) != tuple(v.shape):
        raise ValueError("prob must have the labelled volume's shape")
    pv64 = None
    if pv is not None and pv.dtype == torch.float64:
        # the kernel's per-component maximum is float32; a float64 map keeps its own maximum
        # (float(prob_map[component_mask].max()) in inferencer.py:98), taken below
        pv64, pv = pv, None
    stats = torch.empty(num * 12, dtype=torch.int64, device=dev)
    nat.call("l3u_ccl_stats_b", lab.data_ptr(), None, pv.data_ptr() if pv is not None else None,
             stats.data_ptr(), num, B, D, H, W, lead4, st)
    s = stats.view(num, 12).cpu().numpy().view(np.uint64)
    if min_size > 0:
        keep = s[:, _SIZE] >= min_size
        if not keep.all():
            remap = np.zeros(num + 1, dtype=np.int32)
            remap[1:][keep] = np.arange(1, int(keep.sum()) + 1, dtype=np.int32)
            num = int(keep.sum())
            rm = torch.from_numpy(remap).to(dev)
            if num == 0:   # every component dropped: the remap pass only clears the labels
                stats = torch.empty(12, dtype=torch.int64, device=dev)
                nat.call("l3u_ccl_stats_b", lab.data_ptr(), rm.data_ptr(), None, stats.data_ptr(), 1,
                         B, D, H, W, lead4, st)
                return Components(lab, 0, np.zeros((0, 12), dtype=np.uint64))
            stats = torch.empty(num * 12, dtype=torch.int64, device=dev)
            nat.call("l3u_ccl_stats_b", lab.data_ptr(), rm.data_ptr(),
                     pv.data_ptr() if pv is not None else None, stats.data_ptr(), num, B, D, H, W,
                     lead4, st)
            s = stats.view(num, 12).cpu().numpy().view(np.uint64)
    c = Components(lab, num, s)
    if pv64 is not None:
        m = torch.full((num + 1,), -math.inf, dtype=torch.float64, device=dev)
        m.scatter_reduce_(0, lab.reshape(-1).long(), pv64.reshape(-1), "amax")
        c.pmax64 = m[1:].cpu().numpy()
    return c


def get_connected_components(mask, min_size=0):
    """metrics.py:38-63: (labeled int32 numpy of the mask's shape, num_components); foreground =
    mask != 0; a [B, D, H, W] mask is labelled as one 4-dimensional array, as ndimage.label does."""
    m = np.asarray(mask) if not isinstance(mask, torch.Tensor) else mask
    fg = (m != 0)
    c = label(fg.astype(np.float32) if isinstance(fg, np.ndarray) else fg.float(), 0.5, min_size)
    return c.numpy(), c.num


def _as_components(lab_or_comp):
    if isinstance(lab_or_comp, Components):
        return lab_or_comp
    dev = _device()
    t = lab_or_comp if isinstance(lab_or_comp, torch.Tensor) else torch.from_numpy(
        np.ascontiguousarray(np.asarray(lab_or_comp)))
    B, D, H, W, lead4 = _dims(t.shape)
    t = t.to(device=dev, dtype=torch.int32).contiguous()
    num = int(t.max().item()) if t.numel() else 0
    if num == 0:
        return Components(t, 0, np.zeros((0, 12), dtype=np.uint64))
    stats = torch.empty(num * 12, dtype=torch.int64, device=dev)
    nat.call("l3u_ccl_stats_b", t.data_ptr(), None, None, stats.data_ptr(), num, B, D, H, W, lead4,
             nat.stream())
    return Components(t, num, stats.view(num, 12).cpu().numpy().view(np.uint64))


def _intersections(pc, tc):
    """(num_pred + 1, num_target + 1) int64 overlap counts, row / column 0 zero (metrics.py:153-162)."""
    inter = torch.zeros((pc.num + 1) * (tc.num + 1), dtype=torch.int32, device=pc.labels.device)
    nat.call("l3u_ccl_pairs", pc.labels.data_ptr(), tc.labels.data_ptr(), tc.num, inter.data_ptr(),
             pc.labels.numel(), nat.stream())
    return inter.view(pc.num + 1, tc.num + 1).cpu().numpy().astype(np.int64)


def _sizes0(c):
    out = np.zeros(c.num + 1, dtype=np.int64)
    out[1:] = c.sizes()
    return out


def match_components(pred_labeled, target_labeled, iou_threshold=0.1, distance_threshold_mm=10.0,
                     spacing=(4.0, 4.0, 4.0)):
    """metrics.py:127-213: greedy matching of predicted to target components by IoU or centre
    distance.  Labelled arrays (numpy / device, [D, H, W] or [B, D, H, W]) or Components."""
    pc, tc = _as_components(pred_labeled), _as_components(target_labeled)
    num_pred, num_target = pc.num, tc.num
    if num_pred == 0 or num_target == 0:
        return [], list(range(1, num_pred + 1)), list(range(1, num_target + 1))
    intersection = _intersections(pc, tc)
    pred_sizes, target_sizes = _sizes0(pc), _sizes0(tc)
    union = pred_sizes[:, None] + target_sizes[None, :] - intersection
    iou_matrix = np.divide(intersection, union, out=np.zeros_like(intersection, dtype=np.float32),
                           where=union > 0)
    spacing_arr = np.asarray(spacing, dtype=np.float64)
    pred_centers = pc.centers() * spacing_arr
    target_centers = tc.centers() * spacing_arr
    distance_matrix = np.linalg.norm(pred_centers[:, None, :] - target_centers[None, :, :], axis=2)
    matches = []
    matched_target = np.zeros(num_target, dtype=bool)
    for pid in range(1, num_pred + 1):
        iou_row = iou_matrix[pid, 1:]
        valid = ~matched_target & ((iou_row >= iou_threshold) |
                                   (distance_matrix[pid - 1] <= distance_threshold_mm))
        if not np.any(valid):
            continue
        best = int(np.argmax(np.where(valid, iou_row, -np.inf)))
        matches.append((pid, best + 1))
        matched_target[best] = True
    matched_pred = {p for p, _ in matches}
    return (matches, [i for i in range(1, num_pred + 1) if i not in matched_pred],
            [i for i in range(1, num_target + 1) if not matched_target[i - 1]])


def _squeeze(a):
    if len(a.shape) == 5:
        a = a[:, 0]
    if len(a.shape) == 4 and a.shape[0] == 1:
        a = a[0]
    return a


def _lesion_counts(pc, tc, iou_threshold, distance_threshold_mm, spacing):
    if tc.num == 0:
        return (0, pc.num, 0)
    if pc.num == 0:
        return (0, 0, tc.num)
    m, up, ut = match_components(pc, tc, iou_threshold, distance_threshold_mm, spacing)
    return (len(m), len(up), len(ut))


def calculate_lesion_metrics(pred, target, threshold=0.5, min_size_voxels=0, iou_threshold=0.1,
                             distance_threshold_mm=10.0, spacing=(4.0, 4.0, 4.0)):
    """metrics.py:216-287: lesion-wise recall / precision / f1 and tp / fp / fn counts."""
    pred, target = _squeeze(pred), _squeeze(target)
    pc = label(pred, threshold, min_size_voxels)
    tc = label(target, 0.5, min_size_voxels)
    if tc.num == 0:
        if pc.num == 0:
            return {"recall": 1.0, "precision": 1.0, "f1": 1.0, "tp": 0, "fp": 0, "fn": 0}
        return {"recall": 0.0, "precision": 0.0, "f1": 0.0, "tp": 0, "fp": pc.num, "fn": 0}
    if pc.num == 0:
        return {"recall": 0.0, "precision": 0.0, "f1": 0.0, "tp": 0, "fp": 0, "fn": tc.num}
    tp, fp, fn = _lesion_counts(pc, tc, iou_threshold, distance_threshold_mm, spacing)
    recall = tp / (tp + fn) if (tp + fn) > 0 else 0.0
    precision = tp / (tp + fp) if (tp + fp) > 0 else 0.0
    f1 = 2 * (precision * recall) / (precision + recall) if (precision + recall) > 0 else 0.0
    return {"recall": recall, "precision": precision, "f1": f1, "tp": tp, "fp": fp, "fn": fn}


def calculate_metrics(predictions, labels, threshold=0.5, spacing=(4.0, 4.0, 4.0)):
    """metrics.py:306-404: lesion-wise and voxel-wise (DSC micro / macro) metrics over cases.  The
    voxel counts come from the same device labelling (foreground sizes and overlaps)."""
    pred_list, label_list = _case_list(predictions, "predictions"), _case_list(labels, "labels")
    spacings = _spacing_per_case(spacing, len(pred_list))
    for pred, target in zip(pred_list, label_list):   # shapes first: no device work on a bad list
        _dims(_squeeze(np.asarray(pred)).shape)
        _dims(_squeeze(np.asarray(target)).shape)
    smooth = 1e-6
    tot_tp = tot_fp = tot_fn = 0
    inter_sum = union_sum = 0.0
    per_case = []
    for pred, target, sp in zip(pred_list, label_list, spacings):
        pred, target = _squeeze(np.asarray(pred)), _squeeze(np.asarray(target))
        pc, tc = label(pred, threshold), label(target, 0.5)
        ps, ts = int(pc.sizes().sum()), int(tc.sizes().sum())
        inter = int(_intersections(pc, tc).sum()) if pc.num and tc.num else 0
        inter_sum += inter
        union_sum += ps + ts
        per_case.append((2.0 * inter + smooth) / ((ps + ts) + smooth))
        if tc.num == 0:
            tp, fp, fn = (0, 0 if pc.num == 0 else pc.num, 0)
        elif pc.num == 0:
            tp, fp, fn = (0, 0, tc.num)
        else:
            tp, fp, fn = _lesion_counts(pc, tc, 0.1, 10.0, sp)
        tot_tp += tp
        tot_fp += fp
        tot_fn += fn
    n = len(pred_list)
    dsc_micro = (2.0 * inter_sum + smooth) / (union_sum + smooth)
    dsc_macro = np.mean(per_case) if per_case else 0.0
    recall = tot_tp / (tot_tp + tot_fn) if (tot_tp + tot_fn) > 0 else 0.0
    precision = tot_tp / (tot_tp + tot_fp) if (tot_tp + tot_fp) > 0 else 0.0
    f1 = (2 * precision * recall) / (precision + recall) if (precision + recall) > 0 else 0.0
    return {"lesion_wise_recall": recall, "lesion_wise_precision": precision, "lesion_wise_f1": f1,
            "voxel_wise_dsc_micro": dsc_micro, "voxel_wise_dsc_macro": dsc_macro,
            "fp_per_case": tot_fp / n if n > 0 else 0.0, "tp": tot_tp, "fp": tot_fp, "fn": tot_fn,
            "dsc": dsc_micro, "recall": recall, "precision": precision}


def _case_list(x, what):
    """metrics.py:325-338: a list/tuple, or anything indexable with a leading case axis."""
    if isinstance(x, (list, tuple)):
        return list(x)
    if not (hasattr(x, "shape") and hasattr(x, "__getitem__")):
        raise TypeError(f"{what} must be a list/tuple or array-like object with shape and indexing support")
    return [x[i] for i in range(x.shape[0])]


def _spacing_per_case(spacing, n):
    """metrics.py:290-303: one (z, y, x) spacing per case; DEFAULT_SPACING when malformed."""
    default = (4.0, 4.0, 4.0)
    if n == 0:
        return []
    if isinstance(spacing, np.ndarray):
        spacing = spacing.tolist()
    if isinstance(spacing, (list, tuple)):
        if len(spacing) == 0:
            return [default] * n
        if len(spacing) == n and isinstance(spacing[0], (list, tuple, np.ndarray)):
            return [tuple(map(float, s)) for s in spacing]
        if len(spacing) == 3 and all(isinstance(s, (int, float, np.floating)) for s in spacing):
            return [tuple(map(float, spacing))] * n
    return [default] * n


def extract_bboxes(prob_map, threshold=0.3, min_volume_cc=0.5, spacing=(4.0, 4.0, 4.0),
                   expansion_voxels=0):
    """inferencer.py:62-111 (Inferencer.extract_bboxes, with config["data"]["bbox_expansion_voxels"]
    as an argument): one box per component of (prob >= threshold) with at least
    ceil(min_volume_cc / voxel cc) voxels, expanded and clipped to the volume."""
    pm = prob_map if isinstance(prob_map, torch.Tensor) else np.asarray(prob_map)
    shape = tuple(pm.shape)
    if len(shape) != 3:
        raise ValueError(f"extract_bboxes takes a [D, H, W] probability map, got shape {shape}")
    voxel_volume_cc = spacing[0] * spacing[1] * spacing[2] / 1000.0
    min_voxels = int(np.ceil(min_volume_cc / voxel_volume_cc))
    c = label(pm, threshold, min_voxels, prob=pm)
    out = []
    for cid in range(1, c.num + 1):
        s = c.stats[cid - 1]
        zmin, ymin, xmin = (int(v) for v in s[_MIN])
        zmax, ymax, xmax = (int(v) for v in s[_MAX])
        e = expansion_voxels
        zl, zh = max(0, zmin - e), min(shape[0] - 1, zmax + e)
        yl, yh = max(0, ymin - e), min(shape[1] - 1, ymax + e)
        xl, xh = max(0, xmin - e), min(shape[2] - 1, xmax + e)
        conf = (c.pmax64[cid - 1] if c.pmax64 is not None
                else np.array([int(s[_PMAX])], dtype=np.uint32).view(np.float32)[0])
        out.append({"mask_id": cid,
                    "bbox_voxel": [zl, zh, yl, yh, xl, xh],
                    "bbox_mm": [float(zl * spacing[0]), float(zh * spacing[0]), float(yl * spacing[1]),
                                float(yh * spacing[1]), float(xl * spacing[2]), float(xh * spacing[2])],
                    "volume_cc": float(np.int64(s[_SIZE]) * voxel_volume_cc),
                    "confidence": float(conf)})
    return out


def min_voxels_for(min_volume_cc, spacing):
    """inferencer.py:66-68."""
    return int(math.ceil(min_volume_cc / (spacing[0] * spacing[1] * spacing[2] / 1000.0)))
