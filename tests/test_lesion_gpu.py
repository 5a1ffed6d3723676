"""Device lesion post-processing (light_unet/lesion.py -> csrc/lesion.hip, l3u_ccl_*) against the
reference's own outputs (tests/golden/lesion.npz, made by running light_unet/models/metrics.py)
and against the pinned oracle (oracle/lesion_oracle.py) at larger sizes.  Integer work: labels,
counts, matches and boxes bit-exact; the float metrics equal (same host arithmetic)."""
import numpy as np
import pytest
import torch

from oracle import lesion_oracle as L

pytestmark = pytest.mark.gpu

CC = ["rand30", "rand50", "sparse", "empty", "full", "single", "checker"]


@pytest.mark.parametrize("name", CC)
def test_labels_match_reference(cuda, golden, name):
    from light_unet import lesion
    z = golden("lesion.npz")
    lab, n = lesion.get_connected_components(z[f"cc/{name}/mask"].astype(np.int32))
    assert n == int(z[f"cc/{name}/num"]) and lab.dtype == np.int32
    assert np.array_equal(lab, z[f"cc/{name}/labels"])
    lab5, n5 = lesion.get_connected_components(z[f"cc/{name}/mask"], min_size=5)
    assert n5 == int(z[f"cc/{name}/num_min5"])
    assert np.array_equal(lab5, z[f"cc/{name}/labels_min5"])


@pytest.mark.parametrize("i", range(4))
def test_matching_and_metrics_match_reference(cuda, golden, i):
    from light_unet import lesion
    z = golden("lesion.npz")
    pred, tgt = z[f"lm/{i}/pred"], z[f"lm/{i}/target"]
    for thr in (0.3, 0.5):
        m = lesion.calculate_lesion_metrics(pred, tgt, threshold=thr)
        for k, v in m.items():
            assert v == z[f"lm/{i}/thr{thr}/{k}"].item(), (thr, k)
    m = lesion.calculate_lesion_metrics(pred[None, None], tgt[None, None], threshold=0.3,
                                        min_size_voxels=6, iou_threshold=0.2,
                                        distance_threshold_mm=6.0, spacing=(2.0, 3.0, 4.0))
    for k, v in m.items():
        assert v == z[f"lm/{i}/opts/{k}"].item(), k
    pl, _ = lesion.get_connected_components(pred >= 0.3)
    tl, _ = lesion.get_connected_components(tgt >= 0.5)
    mt, up, ut = lesion.match_components(pl, tl)
    assert np.array_equal(np.array(mt, np.int64).reshape(-1, 2), z[f"lm/{i}/matches"])
    assert list(up) == z[f"lm/{i}/unmatched_pred"].tolist()
    assert list(ut) == z[f"lm/{i}/unmatched_target"].tolist()


def test_batched_arrays_match_reference(cuda, golden):
    """[B, D, H, W] inputs (no host fallback): one 4-dimensional labelling with the batch axis as
    a fourth face neighbour, bit-exact labels / counts vs the reference's ndimage.label; lesion
    metrics on [B, 1, D, H, W] maps and matching of batched and [1, D, H, W] labelled arrays with
    the reference's (b, z, y) centres; calculate_metrics over a [B, 1, D, H, W] array."""
    from light_unet import lesion
    z = golden("lesion.npz")
    lab, n = lesion.get_connected_components(z["b4/cc/mask"].astype(np.int32))
    assert lab.shape == z["b4/cc/labels"].shape and n == int(z["b4/cc/num"])
    assert np.array_equal(lab, z["b4/cc/labels"])
    lab5, n5 = lesion.get_connected_components(z["b4/cc/mask"], min_size=5)
    assert n5 == int(z["b4/cc/num_min5"]) and np.array_equal(lab5, z["b4/cc/labels_min5"])
    pred, tgt = z["b4/lm/pred"], z["b4/lm/target"]
    for thr in (0.3, 0.5):
        for k, v in lesion.calculate_lesion_metrics(pred, tgt, threshold=thr).items():
            assert v == z[f"b4/lm/thr{thr}/{k}"].item(), (thr, k)
    m = lesion.calculate_lesion_metrics(pred[:, 0], tgt[:, 0], threshold=0.3, min_size_voxels=4,
                                        iou_threshold=0.2, distance_threshold_mm=6.0,
                                        spacing=(2.0, 3.0, 4.0))
    for k, v in m.items():
        assert v == z[f"b4/lm/opts/{k}"].item(), k
    pl, _ = lesion.get_connected_components(pred[:, 0] >= 0.3)
    tl, _ = lesion.get_connected_components(tgt[:, 0] >= 0.5)
    for nm, (a, b) in (("b2", (pl, tl)), ("b1", (pl[:1], tl[:1]))):
        mt, up, ut = lesion.match_components(a, b)
        assert np.array_equal(np.array(mt, np.int64).reshape(-1, 2), z[f"b4/match/{nm}/matches"]), nm
        assert list(up) == z[f"b4/match/{nm}/unmatched_pred"].tolist()
        assert list(ut) == z[f"b4/match/{nm}/unmatched_target"].tolist()
    agg = lesion.calculate_metrics(pred, tgt, threshold=0.3)
    for k, v in agg.items():
        assert v == z[f"b4/agg/{k}"].item(), k
    # a larger batched array against the oracle (percolation-level density, 3 items)
    rng = np.random.default_rng(3)
    m4 = rng.random((3, 20, 24, 28)) < 0.3
    lab, n = lesion.get_connected_components(m4)
    labo, no = L.get_connected_components(m4)
    assert n == no and np.array_equal(lab, labo)


def test_calculate_metrics_matches_reference(cuda, golden):
    from light_unet import lesion
    z = golden("lesion.npz")
    preds = [z[f"lm/{i}/pred"] for i in range(4)]
    tgts = [z[f"lm/{i}/target"] for i in range(4)]
    agg = lesion.calculate_metrics(preds, tgts, threshold=0.3,
                                   spacing=[(4.0, 4.0, 4.0), (2.0, 2.0, 2.0), (4.0, 4.0, 4.0), (3.0, 4.0, 5.0)])
    for k, v in agg.items():
        assert v == z[f"agg/{k}"].item(), k


def test_bboxes_match_reference(cuda, golden):
    from light_unet import lesion
    z = golden("lesion.npz")
    bb = lesion.extract_bboxes(z["bb/prob"], 0.3, 0.5, (4.0, 4.0, 4.0), expansion_voxels=2)
    ref = z["bb/boxes"]
    assert len(bb) == ref.shape[0] > 0
    for b, r in zip(bb, ref):
        assert [b["mask_id"]] + b["bbox_voxel"] == r.tolist()
        assert b["bbox_mm"] == [float(v * 4.0) for v in r[1:]]
        assert b["volume_cc"] == z[f"bb/{r[0]}/volume_cc"].item()
        assert b["confidence"] == z[f"bb/{r[0]}/confidence"].item()


@pytest.mark.parametrize("density", [0.1, 0.2, 0.3116, 0.5])
def test_labels_match_oracle_64(cuda, density):
    """64^3 random masks, incl. 3-D site percolation (p ~= 0.3116: components spanning the volume
    through long chains, the worst case for the union-find's contention)."""
    from light_unet import lesion
    m = np.random.default_rng(int(density * 1e4)).random((64, 64, 64)) < density
    lab, n = lesion.get_connected_components(m)
    ref, nr = L.get_connected_components(m)
    assert n == nr and np.array_equal(lab, ref)
    lab2, _ = lesion.get_connected_components(m)
    assert np.array_equal(lab, lab2)      # deterministic


def test_bboxes_match_oracle_ragged(cuda):
    from light_unet import lesion
    rng = np.random.default_rng(3)
    shape = (70, 90, 52)
    zz, yy, xx = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
    p = (rng.random(shape) * 0.05).astype(np.float32)
    for _ in range(30):
        c = [rng.uniform(0, s) for s in shape]
        r = rng.uniform(1.0, 5.0)
        p = np.maximum(p, rng.uniform(0.3, 1.0) * np.exp(
            -((zz - c[0]) ** 2 + (yy - c[1]) ** 2 + (xx - c[2]) ** 2) / (2 * r * r))).astype(np.float32)
    got = lesion.extract_bboxes(torch.from_numpy(p).cuda(), 0.3, 0.5, (2.0, 2.0, 3.0), expansion_voxels=3)
    ref = L.bboxes(p, 0.3, 0.5, (2.0, 2.0, 3.0), expansion_voxels=3)
    assert len(got) == len(ref) > 5
    for g, r in zip(got, ref):
        for k in ("mask_id", "bbox_voxel", "volume_cc", "confidence"):
            assert g[k] == r[k], k


def test_float64_maps_threshold_in_float64(cuda):
    """A float64 probability map (Trainer.validate's prob_map * body_mask) is thresholded in
    float64, as the reference's numpy `pred >= threshold` does (metrics.py:245,
    inferencer.py:64): voxels equal to float32(0.7) = 0.69999998... lie below 0.7 there, so they
    are background; the boxes' confidence is the float64 maximum (inferencer.py:98)."""
    from light_unet import lesion
    rng = np.random.default_rng(11)
    p = rng.random((40, 36, 44)) * 0.6
    blobs = rng.random((40, 36, 44)) < 0.02
    p[blobs] = float(np.float32(0.7))            # just below 0.7 in float64
    hot = rng.random((40, 36, 44)) < 0.01
    p[hot] = 0.7 + rng.random(int(hot.sum())) * 0.3
    assert p.dtype == np.float64
    lab, n = lesion.get_connected_components(p >= 0.7)
    ref, nr = L.get_connected_components(p >= 0.7)
    assert n == nr and np.array_equal(lab, ref)
    tgt = (p >= 0.7).astype(np.float32)
    m = lesion.calculate_lesion_metrics(p, tgt, threshold=0.7)
    assert (m["tp"], m["fp"], m["fn"]) == (nr, 0, 0), m
    got = lesion.extract_bboxes(p, 0.7, 0.0, (4.0, 4.0, 4.0), expansion_voxels=0)
    ref_b = L.bboxes(p, 0.7, 0.0, (4.0, 4.0, 4.0), expansion_voxels=0)
    assert len(got) == len(ref_b) == nr
    for g, r in zip(got, ref_b):
        assert g["bbox_voxel"] == r["bbox_voxel"]
        assert g["confidence"] == float(p[ref == g["mask_id"]].max())
