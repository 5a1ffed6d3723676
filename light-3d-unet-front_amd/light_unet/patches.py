"""Training patches on the MI355X: class-balanced sampling, crop and augmentation of whole case
volumes resident in HBM, mirroring PatchDataset
(light_unet/datasets/patch_dataset.py:17-220).

The reference cuts every patch on the host in a DataLoader worker (numpy crop, scipy rotate /
zoom, numpy noise) and ships it over PCIe.  Here the case volumes are uploaded once, the random
draws stay on the host and are made with the reference's own RNG calls in its order (python
`random` for the flip / rotation axes, numpy's global generator for everything else), and one
launch pair of csrc/augment.hip (l3u_aug_patches) cuts and augments a whole batch from HBM into
the model's [B, 1, pz, py, px] input.  Given the same RNG state, batch element k is the patch the
reference's k-th __getitem__ would return (num_workers = 0 semantics), with scipy's float64
interpolation restated in the kernels (tests/test_patches_gpu.py).
"""
import random

import numpy as np
import torch

from . import _native as nat


class AugDraw:
    """One patch's augmentation, as PatchDataset._augment draws it (patch_dataset.py:156-220)."""
    __slots__ = ("flip_axis", "angle", "rot_axes", "scale", "shift", "noise")

    def __init__(self):
        self.flip_axis, self.angle, self.rot_axes = -1, 0.0, None
        self.scale = self.shift = self.noise = None


def draw_augmentation(aug, patch):
    """The reference's RNG calls of _augment, in order; returns the drawn AugDraw."""
    d = AugDraw()
    if not aug:
        return d
    f = aug.get("random_flip", {})
    if f.get("enabled", False) and np.random.rand() < f.get("prob", 0.5):
        d.flip_axis = int(random.choice(f.get("axes", [0, 1, 2])))
    r = aug.get("random_rotation", {})
    if r.get("enabled", False) and np.random.rand() < r.get("prob", 0.5):
        lo, hi = r.get("angle_range", [-15, 15])
        d.angle = float(np.random.uniform(lo, hi))
        d.rot_axes = tuple(random.choice(r.get("axes", [[0, 1], [0, 2], [1, 2]])))
    s = aug.get("random_scale", {})
    if s.get("enabled", False) and np.random.rand() < s.get("prob", 0.3):
        lo, hi = s.get("scale_range", [0.9, 1.1])
        d.scale = float(np.random.uniform(lo, hi))
    sh = aug.get("intensity_shift", {})
    if sh.get("enabled", False) and np.random.rand() < sh.get("prob", 0.5):
        lo, hi = sh.get("shift_range", [-0.1, 0.1])
        d.shift = float(np.random.uniform(lo, hi))
    g = aug.get("gaussian_noise", {})
    if g.get("enabled", False) and np.random.rand() < g.get("prob", 0.3):
        d.noise = np.random.normal(0, g.get("sigma", 0.01), tuple(patch))
    return d


def _cosdg_sindg(angle):
    """scipy.ndimage.rotate's rotation constants, `special.cosdg(angle), special.sindg(angle)`
    (the cephes degree functions, the reference's own dependency).  Without scipy: exact at
    multiples of 90 degrees, np.cos / np.sin of the radians otherwise (may differ in the last
    ulp)."""
    try:
        from scipy import special
    except ImportError:
        special = None
    if special is not None:
        return float(special.cosdg(angle)), float(special.sindg(angle))
    if angle % 90 == 0:
        k = int(angle // 90) % 4
        return [1.0, 0.0, -1.0, 0.0][k], [0.0, 1.0, 0.0, -1.0][k]
    rad = np.deg2rad(angle)
    return float(np.cos(rad)), float(np.sin(rad))


def aug_param(img_t, lab_t, center, patch, d):
    """The l3u_aug_param record of one patch (crop: patch_dataset.py:136-154; rotate / zoom
    constants computed in float64 exactly as scipy.ndimage.rotate / zoom compute them)."""
    p = nat.AugParam()
    p.image, p.label = img_t.data_ptr(), lab_t.data_ptr()
    sd, sh, sw = img_t.shape
    pz, py, px = patch
    z, y, x = (int(v) for v in center)
    p.z0, p.y0, p.x0 = max(0, z - pz // 2), max(0, y - py // 2), max(0, x - px // 2)
    p.sd, p.sh, p.sw = sd, sh, sw
    p.pz, p.py, p.px = pz, py, px
    p.flip = d.flip_axis
    if d.rot_axes is not None:
        a0, a1 = sorted(int(a) for a in d.rot_axes)
        c, s = _cosdg_sindg(d.angle)
        ic = (np.array([patch[a0], patch[a1]], np.float64) - 1) / 2
        oc = np.array([[c, s], [-s, c]]) @ ic
        off = ic - oc
        p.rot_a0, p.rot_a1 = a0, a1
        p.rot_c, p.rot_s, p.rot_off0, p.rot_off1 = c, s, float(off[0]), float(off[1])
    else:
        p.rot_a0 = p.rot_a1 = -1
    if d.scale is not None:
        zs = [int(round(n * d.scale)) for n in patch]
        p.zoom = 1
        for k in range(3):
            p.zs[k] = zs[k]
            p.zst[k] = (zs[k] - patch[k]) // 2 if zs[k] > patch[k] else 0
            p.zf[k] = (patch[k] - 1) / (zs[k] - 1) if zs[k] != 1 else 1.0
    p.shift_on = 1 if d.shift is not None else 0
    p.shift = d.shift if d.shift is not None else 0.0
    p.noise_on = 1 if d.noise is not None else 0
    return p


class DevicePatchDataset:
    """PatchDataset (patch_dataset.py:17-154) over case volumes resident on the device.

    cases: list of (image, label[, body_mask]) numpy volumes (the NIfTI contents the reference
    loads per item).  Seeding, location sampling (_sample_locations, :74-100) and the per-item
    draws follow the reference; sample_batch(B) returns device tensors [B, 1, *patch_size].
    from_reference() takes a constructed reference PatchDataset instead: its sampled locations
    are kept as they are and each case is read once."""

    def __init__(self, cases, patch_size=(48, 48, 48), lesion_patch_ratio=0.5, augmentation=None,
                 seed=42, device=None, locations=None):
        if not torch.cuda.is_available():
            raise nat.NativeError("DevicePatchDataset needs the ROCm device (no CPU fallback)")
        self.dev = device or torch.device("cuda", torch.cuda.current_device())
        self.patch_size = tuple(int(v) for v in patch_size)
        self.lesion_patch_ratio = lesion_patch_ratio
        self.augmentation = augmentation
        if locations is None:
            random.seed(seed)
            np.random.seed(seed)
        self.vols = []
        for case in cases:
            img, lab = np.asarray(case[0], np.float32), np.asarray(case[1], np.float32)
            if img.shape != lab.shape or img.ndim != 3:
                raise ValueError("image and label must be matching 3D volumes")
            self.vols.append((torch.from_numpy(np.ascontiguousarray(img)).to(self.dev),
                              torch.from_numpy(np.ascontiguousarray(lab)).to(self.dev)))
        if locations is None:
            locations = self._sample_locations(cases)
        self.lesion_locations, self.background_locations = locations
        self.last_draws = []

    @classmethod
    def from_reference(cls, ds, read=None, device=None):
        """The device twin of a constructed reference PatchDataset `ds`: the same cases,
        locations (ds.lesion_locations / background_locations, drawn by its __init__), patch
        size, lesion ratio and augmentation config.  Each case is read ONCE with
        read(path) -> float32 volume (default: `nib.load(path).get_fdata().astype(np.float32)`
        through the nibabel module the reference module imported, patch_dataset.py:129-130)
        and stays in HBM.  Consumes no random numbers."""
        if read is None:
            import sys
            nib = sys.modules[type(ds).__module__].nib

            def read(path):
                return nib.load(path).get_fdata().astype(np.float32)
        cases = [(read(c["image_path"]), read(c["label_path"])) for c in ds.cases]
        return cls(cases, ds.patch_size, ds.lesion_patch_ratio, ds.augmentation, device=device,
                   locations=(list(ds.lesion_locations), list(ds.background_locations)))

    @staticmethod
    def _sample_locations(cases):
        lesion, bg = [], []
        for ci, case in enumerate(cases):
            lab = np.asarray(case[1])
            body = np.asarray(case[2]).astype(bool) if len(case) > 2 and case[2] is not None else None
            lc = np.argwhere(lab > 0)
            if len(lc) > 0:
                for i in np.random.randint(len(lc), size=max(10, len(lc) // 1000)):
                    lesion.append((ci, lc[i]))
            bc = np.argwhere((lab == 0) & body) if body is not None else np.argwhere(lab == 0)
            if len(bc) > 0:
                for i in np.random.randint(len(bc), size=max(10, len(bc) // 5000)):
                    bg.append((ci, bc[i]))
        return lesion, bg

    def __len__(self):
        return len(self.lesion_locations) + len(self.background_locations)

    def _draw_location(self):
        """__getitem__'s location draw (patch_dataset.py:115-124)."""
        if np.random.rand() < self.lesion_patch_ratio and len(self.lesion_locations) > 0:
            return self.lesion_locations[np.random.randint(len(self.lesion_locations))]
        if len(self.background_locations) > 0:
            return self.background_locations[np.random.randint(len(self.background_locations))]
        return self.lesion_locations[np.random.randint(len(self.lesion_locations))]

    def draw_item(self):
        """One __getitem__'s random draws (location, then _augment's), in the reference's order:
        ((case index, centre, AugDraw), its l3u_aug_param record)."""
        case_idx, center = self._draw_location()
        d = draw_augmentation(self.augmentation, self.patch_size)
        img_t, lab_t = self.vols[case_idx]
        return (case_idx, tuple(int(v) for v in center), d), aug_param(img_t, lab_t, center,
                                                                      self.patch_size, d)

    def sample_batch(self, B):
        """B consecutive __getitem__ draws, cut and augmented on the device in one launch pair."""
        items = [self.draw_item() for _ in range(B)]
        self.last_draws = [i[0] for i in items]
        return cut_patches(items, self.patch_size, self.dev)


def cut_patches(items, patch, dev):
    """One l3u_aug_patches launch pair over [(draw, AugParam)] (the records may point into
    different datasets' volumes): device tensors images, labels [B, 1, *patch]."""
    B = len(items)
    arr = (nat.AugParam * B)(*[p for _, p in items])
    prm = torch.frombuffer(bytearray(arr), dtype=torch.uint8).to(dev)
    pz, py, px = patch
    P = pz * py * px
    noise = None
    if any(d.noise is not None for (_, _, d), _ in items):
        nz = np.zeros((B, P), np.float64)
        for k, ((_, _, d), _) in enumerate(items):
            if d.noise is not None:
                nz[k] = d.noise.reshape(-1)
        noise = torch.from_numpy(nz).to(dev)
    tmp = torch.empty(2, B, P, dtype=torch.float32, device=dev)
    out = torch.empty(2, B, 1, pz, py, px, dtype=torch.float32, device=dev)
    nat.call("l3u_aug_patches", prm.data_ptr(), B, pz, py, px,
             noise.data_ptr() if noise is not None else None, tmp[0].data_ptr(),
             tmp[1].data_ptr(), out[0].data_ptr(), out[1].data_ptr(), nat.stream())
    return out[0], out[1]


class DeviceMixedPatchDataset:
    """MixedPatchDataset (patch_dataset.py:223-268) over two DevicePatchDatasets: per item,
    np.random.rand() < fl_ratio picks the FL stream (else DLBCL), the reference's (unused) index
    draw np.random.randint(len(sub)) is made, then the sub-dataset's __getitem__ draws.  The
    per-domain sample counts are kept on `counts` (the reference MixedPatchDataset object when
    built by from_reference, so Trainer.train_epoch reads them there, trainer.py:210-256)."""

    def __init__(self, fl, dlbcl, fl_ratio=0.5, counts=None):
        self.fl, self.dlbcl, self.fl_ratio = fl, dlbcl, fl_ratio
        self.patch_size, self.dev = fl.patch_size, fl.dev
        self.counts = counts if counts is not None else self
        if counts is None:
            self.reset_sample_counts()
        self.last_draws = []

    @classmethod
    def from_reference(cls, ds, read=None, device=None):
        return cls(DevicePatchDataset.from_reference(ds.fl_dataset, read, device),
                   DevicePatchDataset.from_reference(ds.dlbcl_dataset, read, device),
                   ds.fl_ratio, counts=ds)

    def reset_sample_counts(self):
        self.fl_sample_count = 0
        self.dlbcl_sample_count = 0

    def get_sample_counts(self):
        return {"fl_samples": self.fl_sample_count, "dlbcl_samples": self.dlbcl_sample_count,
                "total_samples": self.fl_sample_count + self.dlbcl_sample_count}

    def __len__(self):
        return len(self.fl) + len(self.dlbcl)

    def draw_item(self):
        if np.random.rand() < self.fl_ratio and len(self.fl) > 0:
            self.counts.fl_sample_count += 1
            np.random.randint(len(self.fl))
            return self.fl.draw_item()
        if len(self.dlbcl) > 0:
            self.counts.dlbcl_sample_count += 1
            np.random.randint(len(self.dlbcl))
            return self.dlbcl.draw_item()
        np.random.randint(len(self.fl))
        return self.fl.draw_item()

    def sample_batch(self, B):
        items = [self.draw_item() for _ in range(B)]
        self.last_draws = [i[0] for i in items]
        return cut_patches(items, self.patch_size, self.dev)


class DevicePatchLoader:
    """The training DataLoader of loader.py:9-10 (batch_size, shuffle=True, drop_last=False)
    over a device dataset, with num_workers = 0 semantics: batch k holds the next batch_size
    __getitem__ draws of the process's global numpy / python RNGs (the sampler's index order is
    irrelevant: __getitem__ ignores its index, patch_dataset.py:114-124, :254-261), the last batch
    is ragged, and each epoch takes the two int64 seeds a torch DataLoader iterator draws from
    torch's global generator (the iterator's base seed and RandomSampler's seed), so the torch
    RNG stream after an epoch is the host loader's.  Batches are device tensors
    (images, labels) [b, 1, *patch_size]."""

    def __init__(self, dataset, batch_size):
        self.dataset, self.batch_size = dataset, int(batch_size)

    def __len__(self):
        return (len(self.dataset) + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        torch.empty((), dtype=torch.int64).random_()   # _BaseDataLoaderIter._base_seed
        torch.empty((), dtype=torch.int64).random_()   # RandomSampler's generator seed
        n = len(self.dataset)
        for b0 in range(0, n, self.batch_size):
            yield self.dataset.sample_batch(min(self.batch_size, n - b0))


def device_loader(dataset, batch_size, read=None, device=None):
    """A DevicePatchLoader for a reference PatchDataset / MixedPatchDataset (by duck type:
    MixedPatchDataset carries fl_dataset / dlbcl_dataset)."""
    if hasattr(dataset, "fl_dataset") and hasattr(dataset, "dlbcl_dataset"):
        dd = DeviceMixedPatchDataset.from_reference(dataset, read, device)
    else:
        dd = DevicePatchDataset.from_reference(dataset, read, device)
    return DevicePatchLoader(dd, batch_size)
