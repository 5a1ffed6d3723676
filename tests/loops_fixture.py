"""Reader of tests/golden/loops.npz (made by tests/golden/make_loop_goldens.py from the reference's
own loaders and Trainer): cases, the reference datasets' states, RNG states and expected batches /
scalars.  Shared by tests/test_loops_oracle.py (CPU) and tests/test_reference_loops_gpu.py."""
import json
import os
import random

import numpy as np
import torch

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "loops.npz")


def load():
    z = np.load(PATH, allow_pickle=False)
    meta = json.loads(z["meta"].tobytes().decode())
    return z, meta


def cases(z, meta):
    return {cid: (z[f"case/{cid}/image"].astype(np.float32), z[f"case/{cid}/label"].astype(np.float32))
            for cid in meta["case_ids"]}


def set_rng(z, prefix):
    """Restore the numpy / python / torch global RNG states recorded under prefix."""
    misc = z[prefix + "np_misc"]
    np.random.set_state(("MT19937", z[prefix + "np_keys"].astype(np.uint32), int(misc[0]), int(misc[1]),
                         float(misc[2])))
    pm = z[prefix + "py_misc"]
    random.setstate((int(pm[0]), tuple(int(v) for v in z[prefix + "py_state"]),
                     None if np.isnan(pm[1]) else float(pm[1])))
    torch.set_rng_state(torch.from_numpy(z[prefix + "torch"].copy()))


def rng_matches(z, prefix):
    """The current global RNG states equal the recorded ones (numpy, python, torch)."""
    _, keys, pos, has_g, cached = np.random.get_state()
    misc = z[prefix + "np_misc"]
    ok_np = (np.array_equal(keys, z[prefix + "np_keys"]) and int(pos) == int(misc[0])
             and int(has_g) == int(misc[1]) and (not has_g or float(cached) == float(misc[2])))
    ver, st, _ = random.getstate()
    ok_py = tuple(int(v) for v in z[prefix + "py_state"]) == tuple(st)
    ok_t = np.array_equal(torch.get_rng_state().numpy(), z[prefix + "torch"])
    return ok_np, ok_py, ok_t


def dataset_state(z, meta, prefix):
    """A reference dataset's state: kind 'patch' -> dict(case_ids, lesion, background, patch_size,
    lesion_patch_ratio); kind 'mixed' -> dict(fl=..., dlbcl=..., fl_ratio)."""
    kind = meta[prefix + "kind"]
    if kind == "mixed":
        return {"kind": kind, "fl_ratio": meta[prefix + "fl_ratio"],
                "fl": _patch_state(z, meta, prefix + "fl/"), "dlbcl": _patch_state(z, meta, prefix + "dlbcl/")}
    return dict(_patch_state(z, meta, prefix), kind=kind)


def _patch_state(z, meta, prefix):
    def locs(a):
        return [(int(r[0]), np.array(r[1:], np.int64)) for r in a]
    return {"case_ids": meta[prefix + "case_ids"], "lesion": locs(z[prefix + "lesion"]),
            "background": locs(z[prefix + "background"]), "patch_size": tuple(meta[prefix + "patch_size"]),
            "lesion_patch_ratio": meta[prefix + "lesion_patch_ratio"]}


def batch_sums(x, t):
    x = np.asarray(x, np.float64)
    return np.array([x.shape[0], x.sum(), (x * x).sum(), np.asarray(t, np.float64).sum()])
