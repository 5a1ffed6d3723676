"""Device training patches (light_unet/patches.py -> csrc/augment.hip) against the oracle's
restatement of PatchDataset._extract_patch / _augment (oracle/augment_oracle.py, itself pinned to
scipy.ndimage by tests/test_augment_oracle.py), driven by the same recorded draws.

Tolerances: pure crops / flips / shifts bit-exact; interpolated images |diff| <= 1e-6 (float64
interpolation on both sides, float32 rounding of the same value); labels (nearest neighbour)
may differ only at exact .5 ties: at most 1e-4 of the voxels."""
import numpy as np
import pytest
import torch

from oracle import augment_oracle as A

pytestmark = pytest.mark.gpu

REF_AUG = {"gaussian_noise": {"enabled": True, "prob": 0.3, "sigma": 0.01},
           "intensity_shift": {"enabled": True, "prob": 0.5, "shift_range": [-0.1, 0.1]},
           "random_flip": {"enabled": True, "prob": 0.5, "axes": [0, 1, 2]},
           "random_rotation": {"enabled": True, "prob": 0.5, "angle_range": [-15, 15],
                               "axes": [[0, 1], [0, 2], [1, 2]]},
           "random_scale": {"enabled": True, "prob": 0.3, "scale_range": [0.9, 1.1]}}
ALL_ON = {k: dict(v, prob=1.0) for k, v in REF_AUG.items()}


def _cases(seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for shape in [(60, 70, 52), (50, 44, 64)]:
        img = rng.random(shape, dtype=np.float32) * 0.3
        lab = np.zeros(shape, np.float32)
        zz, yy, xx = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
        for _ in range(4):
            c = [rng.integers(0, s) for s in shape]
            r = rng.uniform(2, 5)
            m = (zz - c[0]) ** 2 + (yy - c[1]) ** 2 + (xx - c[2]) ** 2 <= r * r
            lab[m] = 1.0
            img[m] = rng.uniform(0.6, 1.0)
        out.append((img, lab))
    return out


def _check(ds, cases, imgs, labs, exact=False):
    imgs, labs = imgs.cpu().numpy(), labs.cpu().numpy()
    for k, (ci, center, d) in enumerate(ds.last_draws):
        img, lab = A.extract_patch(cases[ci][0], cases[ci][1], center, ds.patch_size)
        ri, rl = A.augment(img, lab, d, ds.patch_size)
        ri = ri.astype(np.float32)
        if exact:
            assert np.array_equal(imgs[k, 0], ri), k
        else:
            assert np.abs(imgs[k, 0] - ri).max() <= 1e-6, (k, np.abs(imgs[k, 0] - ri).max())
        assert (labs[k, 0] != rl).sum() <= 1e-4 * rl.size, (k, (labs[k, 0] != rl).sum())


def test_patches_crop_only_bit_exact(cuda):
    from light_unet.patches import DevicePatchDataset
    cases = _cases()
    ds = DevicePatchDataset(cases, (48, 48, 48), 0.5, None, seed=1)
    imgs, labs = ds.sample_batch(12)
    assert imgs.shape == (12, 1, 48, 48, 48)
    _check(ds, cases, imgs, labs, exact=True)


@pytest.mark.parametrize("aug,seed", [(ALL_ON, 3), (REF_AUG, 4), (REF_AUG, 5)])
def test_patches_augmented_match_oracle(cuda, aug, seed):
    from light_unet.patches import DevicePatchDataset
    cases = _cases(seed)
    ds = DevicePatchDataset(cases, (48, 48, 48), 0.5, aug, seed=seed)
    for _ in range(2):
        imgs, labs = ds.sample_batch(8)
        _check(ds, cases, imgs, labs)
    if aug is ALL_ON:   # every branch taken
        d = ds.last_draws[0][2]
        assert d.flip_axis >= 0 and d.rot_axes and d.scale and d.shift is not None and d.noise is not None


def test_patches_same_rng_same_batch(cuda):
    from light_unet.patches import DevicePatchDataset
    cases = _cases(7)
    a = DevicePatchDataset(cases, (48, 48, 48), 0.5, REF_AUG, seed=9).sample_batch(6)
    b = DevicePatchDataset(cases, (48, 48, 48), 0.5, REF_AUG, seed=9).sample_batch(6)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
