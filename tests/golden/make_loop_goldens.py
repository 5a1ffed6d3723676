"""Golden fixtures for the training-patch pipeline and the Trainer loops, made by the REFERENCE's
own code (VERDICT r3 "Next round" item 5).

Run here (where /root/reference exists) with
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_loop_goldens.py
It imports the reference package itself (`light_unet.datasets.loader`, `.patch_dataset`,
`light_unet.core.trainer`, unmodified, from /root/reference) with two stand-ins for modules that
are absent from this image and that only do I/O around the path:
  * `nibabel`: `load(path).get_fdata()` returns the float64 array of a .npy payload (the reference
    reads NIfTI volumes, patch_dataset.py:79,127-128; its arithmetic starts at that array);
  * `torch.utils.tensorboard.SummaryWriter`: records every `add_scalar(tag, value, step)`
    (trainer.py:11,156; the loops' logging is part of what is pinned).
and one configuration choice: the training DataLoader is built with num_workers = 0
(`loader._create_train_loader`, loader.py:9-10; the reference uses 16 worker processes, whose
reseeded numpy streams no single-process loader reproduces -- INTEGRATION.md), everything else
(`get_data_loader`, `PatchDataset.__init__` / `_sample_locations` / `__getitem__` /
`_extract_patch` / `_augment` with scipy's rotate / zoom, `MixedPatchDataset`, `Trainer.__init__`,
`train_epoch`, `_train_epoch_step_based`) is the reference code running on CPU.

tests/golden/loops.npz holds, as data only:
  * the synthetic cases (2 FL ids 0001-0002, 2 DLBCL ids 1001-1002; image float32, label uint8);
  * per loader mode (standard, fl_epoch_plus_dlbcl's FL and DLBCL loaders, probabilistic): the
    state each reference dataset was built with (case ids in order, sampled lesion / background
    locations, patch size, lesion ratio, fl_ratio), the numpy / python / torch RNG states just
    before the epoch, the first K batches (images, labels), a checksum row per batch of the whole
    epoch, the RNG states after it and the mixed dataset's domain counts;
  * per Trainer mode: the reference model's initial state_dict (Trainer.__init__ under the config
    seed), the RNG states just before train_epoch(0), the datasets' states, and for epochs 0 and 1
    every recorded scalar (tag, step, value) and the returned average loss.
The JSON part (configs, tag lists) is stored as a uint8 array `meta`.
"""
import json
import os
import random
import sys
import tempfile
import types

sys.dont_write_bytecode = True

import numpy as np
import torch

REF = os.environ.get("L3U_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))
PATCH = (16, 16, 16)
BATCH = 3
K_BATCHES = 4
CASES = {"0001": (24, 28, 20), "0002": (20, 24, 28), "1001": (28, 20, 24), "1002": (24, 24, 24)}
AUG = {"gaussian_noise": {"enabled": True, "mean": 0.0, "prob": 0.3, "sigma": 0.01},
       "intensity_shift": {"enabled": True, "prob": 0.5, "shift_range": [-0.1, 0.1]},
       "random_flip": {"axes": [0, 1, 2], "enabled": True, "prob": 0.5},
       "random_rotation": {"angle_range": [-15, 15], "axes": [[0, 1], [0, 2], [1, 2]],
                           "enabled": True, "prob": 0.5},
       "random_scale": {"enabled": True, "prob": 0.3, "scale_range": [0.9, 1.1]}}


# ---------------------------------------------------------------- stand-ins for absent I/O modules
class _Img:
    def __init__(self, a):
        self._a = a

    def get_fdata(self):
        return np.asarray(self._a, dtype=np.float64)


def _install_stubs():
    nib = types.ModuleType("nibabel")
    nib.load = lambda path: _Img(np.load(str(path), allow_pickle=False))
    sys.modules["nibabel"] = nib
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:
        log = []

        def __init__(self, *a, **k):
            pass

        def add_scalar(self, tag, value, step):
            SummaryWriter.log.append((str(tag), int(step), float(value)))

        def close(self):
            pass
    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    return SummaryWriter


def _write_cases(root):
    """Synthetic PET-like cases under the reference's layout (utils.py:176-214: images/<id>_0000,
    labels/<id>); .npy payloads behind .nii.gz names (read by the nibabel stand-in)."""
    rng = np.random.default_rng(2024)
    os.makedirs(os.path.join(root, "data", "images"))
    os.makedirs(os.path.join(root, "data", "labels"))
    os.makedirs(os.path.join(root, "splits"))
    vols = {}
    for cid, shape in CASES.items():
        img = (rng.random(shape) * 0.3).astype(np.float32)
        lab = np.zeros(shape, np.float32)
        zz, yy, xx = np.meshgrid(*[np.arange(s) for s in shape], indexing="ij")
        for _ in range(2):
            c = [rng.integers(4, s - 4) for s in shape]
            m = (zz - c[0]) ** 2 + (yy - c[1]) ** 2 + (xx - c[2]) ** 2 <= rng.uniform(2, 4) ** 2
            lab[m] = 1.0
            img[m] = rng.uniform(0.6, 1.0, size=int(m.sum())).astype(np.float32)
        for sub, name, arr in (("images", f"{cid}_0000.nii.gz", img), ("labels", f"{cid}.nii.gz", lab)):
            with open(os.path.join(root, "data", sub, name), "wb") as f:
                np.save(f, arr)
        vols[cid] = (img, lab)
    ids = list(CASES)
    for split in ("train_list.txt", "val_list.txt"):
        with open(os.path.join(root, "splits", split), "w") as f:
            f.write("\n".join(ids) + "\n")
    return vols


def _config(root, mode):
    mixed = {"enabled": mode != "standard", "mode": mode if mode != "standard" else "probabilistic",
             "fl_ratio": 0.6, "dlbcl_steps": None, "dlbcl_steps_ratio": 1.0, "dlbcl_ratio": 0.5}
    return {
        "experiment": {"seed": 7},
        "data_dir": os.path.join(root, "data"), "splits_dir": os.path.join(root, "splits"),
        "data": {"patch_size": list(PATCH), "body_mask": {"enabled": False},
                 "domains": {"fl_prefix_max": 122, "dlbcl_prefix_min": 1000, "dlbcl_prefix_max": 1422},
                 "spacing": {"target": [4.0, 4.0, 4.0]}},
        "augmentation": AUG,
        "model": {"output_channels": 1, "start_channels": 8, "encoder_channels": [8, 16, 32, 64],
                  "use_depthwise_separable": True, "use_grouped_conv": True, "groups": 8,
                  "dropout_p": 0.1, "use_dropout": False},
        "loss": {"name": "FocalTverskyLoss", "alpha": 0.7, "beta": 0.3, "gamma": 0.75,
                 "use_combined_loss": False},
        "training": {"batch_size": BATCH, "learning_rate": 1e-4, "weight_decay": 1e-5,
                     "scheduler": {"name": "CosineAnnealingLR", "T_max": 10, "eta_min": 1e-6},
                     "class_balanced_sampling": {"enabled": True, "lesion_patch_ratio": 0.5},
                     "mixed_domains": mixed},
        "output": {"log_dir": os.path.join(root, "out", "logs"),
                   "tensorboard_dir": os.path.join(root, "out", "tb"),
                   "checkpoint_dir": os.path.join(root, "out", "ckpt")},
    }


def seed_all(s):
    random.seed(s)
    np.random.seed(s)
    torch.manual_seed(s)


def rng_state():
    """(numpy keys, numpy pos / has_gauss / cached_gaussian, python state, torch state) as arrays."""
    _, keys, pos, has_g, cached = np.random.get_state()
    ver, pystate, gnext = random.getstate()
    return {"np_keys": np.asarray(keys, np.uint32),
            "np_misc": np.array([pos, has_g, cached], np.float64),
            "py_state": np.asarray(pystate, np.uint64),
            "py_misc": np.array([ver, np.nan if gnext is None else gnext], np.float64),
            "torch": torch.get_rng_state().numpy().copy()}


def _put(out, prefix, d):
    for k, v in d.items():
        out[f"{prefix}{k}"] = v


def _dataset_state(ds, prefix, out, meta):
    """What the device twin of a reference PatchDataset is built from."""
    ids = [c["case_id"] for c in ds.cases]
    les = ds.lesion_locations
    bg = ds.background_locations
    out[prefix + "lesion"] = np.array([[ci, *map(int, c)] for ci, c in les], np.int32).reshape(-1, 4)
    out[prefix + "background"] = np.array([[ci, *map(int, c)] for ci, c in bg], np.int32).reshape(-1, 4)
    meta[prefix + "case_ids"] = ids
    meta[prefix + "patch_size"] = [int(v) for v in ds.patch_size]
    meta[prefix + "lesion_patch_ratio"] = float(ds.lesion_patch_ratio)


def _describe(ds, prefix, out, meta):
    if hasattr(ds, "fl_dataset"):
        meta[prefix + "kind"] = "mixed"
        meta[prefix + "fl_ratio"] = float(ds.fl_ratio)
        _dataset_state(ds.fl_dataset, prefix + "fl/", out, meta)
        _dataset_state(ds.dlbcl_dataset, prefix + "dlbcl/", out, meta)
    else:
        meta[prefix + "kind"] = "patch"
        _dataset_state(ds, prefix, out, meta)


def _epoch(loader, prefix, out):
    """Iterate one epoch: first K batches stored, one checksum row per batch."""
    sums = []
    for b, (x, t) in enumerate(loader):
        x, t = x.numpy().astype(np.float64), t.numpy()
        sums.append([x.shape[0], x.sum(), (x * x).sum(), t.sum()])
        if b < K_BATCHES:
            out[f"{prefix}x{b}"] = x.astype(np.float32)
            out[f"{prefix}t{b}"] = t.astype(np.uint8)
    out[prefix + "sums"] = np.array(sums, np.float64)


def main():
    Writer = _install_stubs()
    sys.path.insert(0, REF)
    from light_unet.datasets import loader as L
    import light_unet.datasets.patch_dataset as PD   # noqa: F401  (the module the loaders use)
    from torch.utils.data import DataLoader

    def _create_train_loader(dataset, batch_size, shuffle=True):   # loader.py:9-10, 0 workers
        return DataLoader(dataset, batch_size=batch_size, shuffle=shuffle, num_workers=0)
    L._create_train_loader = _create_train_loader
    from light_unet.core import trainer as TR

    out, meta = {}, {"patch": list(PATCH), "batch": BATCH, "k_batches": K_BATCHES}
    with tempfile.TemporaryDirectory() as root:
        vols = _write_cases(root)
        for cid, (img, lab) in vols.items():
            out[f"case/{cid}/image"] = img
            out[f"case/{cid}/label"] = lab.astype(np.uint8)
        meta["case_ids"] = list(vols)
        # ---- the training loaders (get_data_loader, loader.py:99-113), one epoch each
        for mode in ("standard", "fl_epoch_plus_dlbcl", "probabilistic"):
            cfg = _config(root, mode)
            seed_all(5)
            r = L.get_data_loader(cfg["data_dir"], os.path.join(cfg["splits_dir"], "train_list.txt"),
                                  cfg, is_train=True)
            assert r["mode"] == mode
            names = ["fl_loader", "dlbcl_loader"] if mode == "fl_epoch_plus_dlbcl" else ["train_loader"]
            meta[f"loader/{mode}/loaders"] = names
            for nm in names:
                _describe(r[nm].dataset, f"loader/{mode}/{nm}/", out, meta)
            _put(out, f"loader/{mode}/rng_before/", rng_state())
            for nm in names:
                meta[f"loader/{mode}/{nm}/len"] = len(r[nm])
                _epoch(r[nm], f"loader/{mode}/{nm}/", out)
            _put(out, f"loader/{mode}/rng_after/", rng_state())
            if "train_dataset" in r:
                meta[f"loader/{mode}/counts"] = r["train_dataset"].get_sample_counts()
        # ---- the Trainer loops (trainer.py:208-347) on the reference model, two epochs
        for mode in ("standard", "fl_epoch_plus_dlbcl", "probabilistic"):
            cfg = _config(root, mode)
            seed_all(5)
            t = TR.Trainer(cfg)
            assert str(t.device) == "cpu"
            pre = f"trainer/{mode}/"
            meta[pre + "config"] = cfg
            for k, v in t.model.state_dict().items():
                out[pre + "init/" + k] = v.detach().numpy().copy()
            names = (["fl_loader", "dlbcl_loader"] if t.use_step_based_mixed else ["train_loader"])
            meta[pre + "loaders"] = names
            for nm in names:
                _describe(getattr(t, nm).dataset, pre + nm + "/", out, meta)
            _put(out, pre + "rng_before/", rng_state())
            for epoch in (0, 1):
                Writer.log.clear()
                avg = t.train_epoch(epoch)
                meta[pre + f"epoch{epoch}/return"] = float(avg)
                meta[pre + f"epoch{epoch}/scalars"] = list(Writer.log)
            _put(out, pre + "rng_after/", rng_state())
            for k, v in t.model.state_dict().items():
                out[pre + "final/" + k] = v.detach().numpy().copy()
            print(mode, "epoch returns", meta[pre + "epoch0/return"], meta[pre + "epoch1/return"],
                  "steps", sum(1 for s in meta[pre + "epoch0/scalars"] if s[0] == "Loss/train_step"))
    out["meta"] = np.frombuffer(json.dumps(meta).encode(), np.uint8)
    np.savez_compressed(os.path.join(OUT, "loops.npz"), **out)
    print("wrote", os.path.join(OUT, "loops.npz"), os.path.getsize(os.path.join(OUT, "loops.npz")), "bytes")


if __name__ == "__main__":
    main()
