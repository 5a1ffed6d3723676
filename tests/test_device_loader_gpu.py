"""l3u_plugin.install(device_patches=True): get_data_loader's training loaders cut and augment
their patches on the device (light_unet/patches.py DevicePatchLoader) with the host loaders'
batches.

The reference's datasets need nibabel (patch_dataset.py:7), absent here, so a stand-in package
with the reference's module layout is used (as tests/test_plugin.py does): a PatchDataset /
MixedPatchDataset / loader factory whose __getitem__ makes the reference's RNG calls in order and
whose image work is the oracle's (oracle/augment_oracle.py, pinned to scipy), and a
`nib.load(path).get_fdata()` over .npy files.  Host side: torch DataLoader(shuffle=True,
num_workers=0).  Device side: the same factories after install().  Compared per mode (standard,
fl_epoch_plus_dlbcl, probabilistic): batch count and shapes (ragged last batch), images
<= 1e-6, labels (nearest-neighbour ties) <= 1e-4 of the voxels, the RNG states after the epoch
(numpy, python, torch), the mixed dataset's domain counts; and Trainer.train_epoch (the
fast_step loop) consuming both loaders gives the same per-step losses.  This test covers the
install() plumbing against a stand-in package; the draw ORDER and the batches themselves are
pinned to the reference's own loaders by tests/test_reference_loops_gpu.py (and, on CPU,
tests/test_loops_oracle.py) over reference-generated fixtures (tests/golden/loops.npz)."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-3d-unet-front_amd")

PATCH_DATASET = '''
import random
import numpy as np
import torch
from torch.utils.data import Dataset
from oracle import augment_oracle as A
from l3u_amd.patches import AugDraw


class _Img:
    def __init__(self, a):
        self.a = a

    def get_fdata(self):
        return self.a.astype(np.float64)


class nib:   # nibabel stand-in: the cases are .npy files
    @staticmethod
    def load(path):
        return _Img(np.load(path))


class PatchDataset(Dataset):
    def __init__(self, data_dir, split_file, patch_size=(48, 48, 48), lesion_patch_ratio=0.5,
                 augmentation=None, seed=42, domain_config=None, body_mask_config=None):
        self.patch_size, self.lesion_patch_ratio, self.augmentation = patch_size, lesion_patch_ratio, augmentation
        random.seed(seed)
        np.random.seed(seed)
        dom = (domain_config or {}).get("domain", "fl")
        ids = [l.strip() for l in open(split_file) if l.strip() and l.startswith(dom)]
        self.cases = [{"case_id": i, "image_path": f"{data_dir}/{i}_img.npy",
                       "label_path": f"{data_dir}/{i}_lab.npy"} for i in ids]
        self.lesion_locations, self.background_locations = [], []
        for ci, c in enumerate(self.cases):
            lab = nib.load(c["label_path"]).get_fdata()
            lc = np.argwhere(lab > 0)
            if len(lc) > 0:
                for i in np.random.randint(len(lc), size=max(10, len(lc) // 1000)):
                    self.lesion_locations.append((ci, lc[i]))
            bc = np.argwhere(lab == 0)
            if len(bc) > 0:
                for i in np.random.randint(len(bc), size=max(10, len(bc) // 5000)):
                    self.background_locations.append((ci, bc[i]))

    def __len__(self):
        return len(self.lesion_locations) + len(self.background_locations)

    def __getitem__(self, idx):
        if np.random.rand() < self.lesion_patch_ratio and len(self.lesion_locations) > 0:
            ci, center = self.lesion_locations[np.random.randint(len(self.lesion_locations))]
        elif len(self.background_locations) > 0:
            ci, center = self.background_locations[np.random.randint(len(self.background_locations))]
        else:
            ci, center = self.lesion_locations[np.random.randint(len(self.lesion_locations))]
        c = self.cases[ci]
        image = nib.load(c["image_path"]).get_fdata().astype(np.float32)
        label = nib.load(c["label_path"]).get_fdata().astype(np.float32)
        img, lab = A.extract_patch(image, label, center, self.patch_size)
        d, a = AugDraw(), self.augmentation or {}
        if a.get("random_flip", {}).get("enabled") and np.random.rand() < a["random_flip"]["prob"]:
            d.flip_axis = int(random.choice(a["random_flip"]["axes"]))
        if a.get("random_rotation", {}).get("enabled") and np.random.rand() < a["random_rotation"]["prob"]:
            d.angle = float(np.random.uniform(*a["random_rotation"]["angle_range"]))
            d.rot_axes = tuple(random.choice(a["random_rotation"]["axes"]))
        if a.get("random_scale", {}).get("enabled") and np.random.rand() < a["random_scale"]["prob"]:
            d.scale = float(np.random.uniform(*a["random_scale"]["scale_range"]))
        if a.get("intensity_shift", {}).get("enabled") and np.random.rand() < a["intensity_shift"]["prob"]:
            d.shift = float(np.random.uniform(*a["intensity_shift"]["shift_range"]))
        if a.get("gaussian_noise", {}).get("enabled") and np.random.rand() < a["gaussian_noise"]["prob"]:
            d.noise = np.random.normal(0, a["gaussian_noise"]["sigma"], tuple(self.patch_size))
        img, lab = A.augment(img, lab, d, self.patch_size)
        return (torch.from_numpy(img.astype(np.float32)).unsqueeze(0),
                torch.from_numpy(lab.astype(np.float32)).unsqueeze(0))


class MixedPatchDataset(Dataset):
    def __init__(self, data_dir, split_file, patch_size=(48, 48, 48), lesion_patch_ratio=0.5,
                 augmentation=None, seed=42, domain_config=None, fl_ratio=0.5, body_mask_config=None):
        self.fl_ratio = fl_ratio
        self.fl_dataset = PatchDataset(data_dir, split_file, patch_size, lesion_patch_ratio,
                                       augmentation, seed, {"domain": "fl"})
        self.dlbcl_dataset = PatchDataset(data_dir, split_file, patch_size, lesion_patch_ratio,
                                          augmentation, seed + 1, {"domain": "dlbcl"})
        self.reset_sample_counts()

    def __len__(self):
        return len(self.fl_dataset) + len(self.dlbcl_dataset)

    def __getitem__(self, idx):
        if np.random.rand() < self.fl_ratio and len(self.fl_dataset) > 0:
            self.fl_sample_count += 1
            return self.fl_dataset[np.random.randint(len(self.fl_dataset))]
        elif len(self.dlbcl_dataset) > 0:
            self.dlbcl_sample_count += 1
            return self.dlbcl_dataset[np.random.randint(len(self.dlbcl_dataset))]
        return self.fl_dataset[np.random.randint(len(self.fl_dataset))]

    def reset_sample_counts(self):
        self.fl_sample_count = 0
        self.dlbcl_sample_count = 0

    def get_sample_counts(self):
        return {"fl_samples": self.fl_sample_count, "dlbcl_samples": self.dlbcl_sample_count,
                "total_samples": self.fl_sample_count + self.dlbcl_sample_count}
'''

LOADER = '''
from torch.utils.data import DataLoader
from .patch_dataset import PatchDataset, MixedPatchDataset


def _create_train_loader(dataset, batch_size, shuffle=True):
    return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, num_workers=0)


def get_data_loader(data_dir, split_file, config, is_train=True):
    aug, ps, seed, bs = config["augmentation"], config["patch_size"], config["seed"], config["batch_size"]
    mode = config["mode"]
    if mode == "fl_epoch_plus_dlbcl":
        fl = PatchDataset(data_dir, split_file, ps, 0.5, aug, seed, {"domain": "fl"})
        dl = PatchDataset(data_dir, split_file, ps, 0.5, aug, seed + 1, {"domain": "dlbcl"})
        return {"mode": mode, "fl_loader": _create_train_loader(fl, bs),
                "dlbcl_loader": _create_train_loader(dl, bs)}
    if mode == "probabilistic":
        ds = MixedPatchDataset(data_dir, split_file, ps, 0.5, aug, seed, None, 0.6)
        return {"mode": mode, "train_loader": _create_train_loader(ds, bs), "train_dataset": ds}
    ds = PatchDataset(data_dir, split_file, ps, 0.5, aug, seed, None)
    return {"mode": "standard", "train_loader": _create_train_loader(ds, bs)}
'''

SCRIPT = '''
import importlib.util, random, sys
import numpy as np
import torch
sys.path[:0] = [TMP, ROOT]
spec = importlib.util.spec_from_file_location("l3u_plugin", PKG + "/l3u_plugin.py")
plug = importlib.util.module_from_spec(spec); spec.loader.exec_module(plug)
plug.load()
from light_unet.datasets import loader as L

AUG = {"gaussian_noise": {"enabled": True, "prob": 0.3, "sigma": 0.01},
       "intensity_shift": {"enabled": True, "prob": 0.5, "shift_range": [-0.1, 0.1]},
       "random_flip": {"enabled": True, "prob": 0.5, "axes": [0, 1, 2]},
       "random_rotation": {"enabled": True, "prob": 0.5, "angle_range": [-15, 15],
                           "axes": [[0, 1], [0, 2], [1, 2]]},
       "random_scale": {"enabled": True, "prob": 0.3, "scale_range": [0.9, 1.1]}}


def seed_all(s):
    random.seed(s); np.random.seed(s); torch.manual_seed(s)


def rng_state():
    return (np.random.get_state()[1].tobytes(), np.random.get_state()[2], random.getstate(),
            torch.get_rng_state().numpy().tobytes())


def epoch(mode):
    seed_all(5)
    r = L.get_data_loader(TMP + "/data", TMP + "/data/train_list.txt",
                          {"augmentation": AUG, "patch_size": (32, 32, 32), "seed": 7,
                           "batch_size": 3, "mode": mode})
    out = {}
    for k in ("train_loader", "fl_loader", "dlbcl_loader"):
        if k in r:
            out[k] = [(x.cpu().numpy(), t.cpu().numpy()) for x, t in r[k]]
            out[k + "_len"] = len(r[k])
    if "train_dataset" in r:
        out["counts"] = r["train_dataset"].get_sample_counts()
    out["rng"] = rng_state()
    return out, r


host = {m: epoch(m)[0] for m in ("standard", "fl_epoch_plus_dlbcl", "probabilistic")}
done = plug.install(fast_step=True, device_patches=True)
assert done["light_unet.datasets.loader"] == ["_create_train_loader"]
for mode, h in host.items():
    d, res = epoch(mode)
    assert d["rng"] == h["rng"], mode
    assert d.get("counts") == h.get("counts"), (mode, d.get("counts"), h.get("counts"))
    for k in ("train_loader", "fl_loader", "dlbcl_loader"):
        if k not in h:
            continue
        assert type(res[k]).__name__ == "DevicePatchLoader"
        assert d[k + "_len"] == h[k + "_len"] == len(h[k]) == len(d[k]), (mode, k)
        for (xd, td), (xh, th) in zip(d[k], h[k]):
            assert xd.shape == xh.shape and td.shape == th.shape, (xd.shape, xh.shape)
            assert np.abs(xd - xh).max() <= 1e-6, (mode, k, np.abs(xd - xh).max())
            assert (td != th).sum() <= 1e-4 * th.size, (mode, k, (td != th).sum())
    print("MODE OK", mode, h.get("train_loader_len", h.get("fl_loader_len")))

# Trainer.train_epoch (fast_step loop) on the device loader and on the host loader: same losses
fast = sys.modules["l3u_amd.fast_trainer"]
Net = sys.modules["l3u_amd.models.unet3d"].Lightweight3DUNet
FTL = sys.modules["l3u_amd.models.losses"].FocalTverskyLoss


class W:
    def add_scalar(self, *a):
        pass


def trainer(loader_fn):
    seed_all(5)
    class T:
        pass
    t = T()
    torch.manual_seed(42)
    t.model = Net(encoder_channels=[8, 16, 32, 64], dropout_p=0.0).cuda()
    t.criterion = FTL()
    t.optimizer = torch.optim.AdamW(t.model.parameters(), lr=1e-4, weight_decay=1e-5)
    t.writer, t.use_step_based_mixed, t.use_mixed_training, t.train_dataset = W(), False, False, None
    t.train_loader = loader_fn()
    losses = []
    orig = fast.FastLoop.losses
    fast.FastLoop.losses = lambda self: losses.extend(orig(self)) or orig(self)
    try:
        avg = fast.train_epoch(t, 0)
    finally:
        fast.FastLoop.losses = orig
    return avg, losses


def mk(dev):
    ds = sys.modules["light_unet.datasets.patch_dataset"].PatchDataset(
        TMP + "/data", TMP + "/data/train_list.txt", (32, 32, 32), 0.5, AUG, 7, None)
    return L._create_train_loader(ds, 3) if dev else L._create_train_loader._l3u_reference(ds, 3)


ad, ld = trainer(lambda: mk(True))
ah, lh = trainer(lambda: mk(False))
assert len(ld) == len(lh) > 3 and all(np.isfinite(ld)), (ld, lh)
assert np.allclose(ld, lh, rtol=1e-5, atol=1e-6), (ld, lh)
print("TRAIN OK", len(ld), ad, ah)
'''


def _write_standin(tmp):
    import numpy as np
    base = tmp / "light_unet"
    for d in ("models", "core", "datasets"):
        (base / d).mkdir(parents=True)
        (base / d / "__init__.py").write_text("")
    (base / "__init__.py").write_text("")
    (base / "utils.py").write_text("def sliding_window_inference_3d(*a, **k):\n    return 'reference'\n")
    (base / "models" / "unet3d.py").write_text("class Lightweight3DUNet:\n    pass\n")
    (base / "models" / "losses.py").write_text(
        "class FocalTverskyLoss:\n    pass\n\ndef get_loss_function(cfg):\n    return None\n")
    (base / "core" / "trainer.py").write_text(
        "class Trainer:\n    def train_epoch(self, e):\n        return 'reference'\n"
        "    def _train_epoch_step_based(self, e):\n        return 'reference'\n")
    (base / "datasets" / "patch_dataset.py").write_text(PATCH_DATASET)
    (base / "datasets" / "loader.py").write_text(LOADER)
    data = tmp / "data"
    data.mkdir()
    rng = np.random.default_rng(0)
    ids = []
    for k, shape in enumerate([(40, 44, 36), (36, 40, 48), (44, 36, 40)]):
        for dom in ("fl", "dlbcl"):
            img = (rng.random(shape) * 0.3).astype(np.float32)
            lab = np.zeros(shape, np.float32)
            zz, yy, xx = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
            for _ in range(3):
                c = [rng.integers(4, s - 4) for s in shape]
                m = (zz - c[0]) ** 2 + (yy - c[1]) ** 2 + (xx - c[2]) ** 2 <= rng.uniform(2, 5) ** 2
                lab[m] = 1.0
                img[m] = rng.uniform(0.6, 1.0)
            cid = f"{dom}{k:03d}"
            np.save(data / f"{cid}_img.npy", img)
            np.save(data / f"{cid}_lab.npy", lab)
            ids.append(cid)
    (data / "train_list.txt").write_text("\n".join(ids) + "\n")


def test_device_loaders_match_host_loaders(cuda, tmp_path):
    _write_standin(tmp_path)
    script = f"TMP, ROOT, PKG = {str(tmp_path)!r}, {ROOT!r}, {PKG!r}\n" + textwrap.dedent(SCRIPT)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=600,
                       cwd=str(tmp_path))
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert r.stdout.count("MODE OK") == 3 and "TRAIN OK" in r.stdout, r.stdout
