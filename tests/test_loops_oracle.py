"""CPU: the host half of the device training loaders (light_unet/patches.py: the reference's RNG
calls in order, the location draw, the mixed-domain pick, DevicePatchLoader's batching and torch
seed draws) driven with the image math of the oracle (oracle/augment_oracle.py), against batches
made by the REFERENCE's own get_data_loader / PatchDataset / MixedPatchDataset
(tests/golden/loops.npz, tests/golden/make_loop_goldens.py): the first batches elementwise, a
checksum of every batch of the epoch, and the numpy / python / torch RNG states after it.  This
pins the draw order that round 3 could only restate (missing item 2)."""
import numpy as np
import pytest
import torch

import loops_fixture as LF
from light_unet import patches as LP
from oracle import augment_oracle as A


class _HostPatchDataset(LP.DevicePatchDataset):
    """DevicePatchDataset's draw logic with CPU volumes; sample_batch cuts with the oracle."""

    def __init__(self, st, vols, aug):
        self.dev = torch.device("cpu")
        self.patch_size = tuple(st["patch_size"])
        self.lesion_patch_ratio = st["lesion_patch_ratio"]
        self.augmentation = aug
        self.np_vols = [vols[cid] for cid in st["case_ids"]]
        self.vols = [(torch.from_numpy(i), torch.from_numpy(l)) for i, l in self.np_vols]
        self.lesion_locations, self.background_locations = st["lesion"], st["background"]
        self.last_draws = []

    def cut(self, draw):
        ci, center, d = draw
        img, lab = self.np_vols[ci]
        ip, lp = A.extract_patch(img, lab, center, self.patch_size)
        return A.augment(ip, lp, d, self.patch_size)

    def sample_batch(self, B):
        items = [self.draw_item() for _ in range(B)]
        out = [self.cut(d) for d, _ in items]
        return (torch.from_numpy(np.stack([o[0] for o in out])[:, None].astype(np.float32)),
                torch.from_numpy(np.stack([o[1] for o in out])[:, None].astype(np.float32)))


class _HostMixed(LP.DeviceMixedPatchDataset):
    """DeviceMixedPatchDataset's per-item domain pick; each item cut by its sub-dataset."""

    def sample_batch(self, B):
        out = []
        for _ in range(B):
            fl_before, dl_before = self.counts.fl_sample_count, self.counts.dlbcl_sample_count
            draw, _ = self.draw_item()
            ds = self.dlbcl if self.counts.dlbcl_sample_count != dl_before else self.fl
            assert self.counts.fl_sample_count != fl_before or ds is self.dlbcl or len(self.dlbcl) == 0
            out.append(ds.cut(draw))
        return (torch.from_numpy(np.stack([o[0] for o in out])[:, None].astype(np.float32)),
                torch.from_numpy(np.stack([o[1] for o in out])[:, None].astype(np.float32)))


def host_dataset(st, vols, aug):
    if st["kind"] == "mixed":
        return _HostMixed(_HostPatchDataset(st["fl"], vols, aug), _HostPatchDataset(st["dlbcl"], vols, aug),
                          st["fl_ratio"])
    return _HostPatchDataset(st, vols, aug)


@pytest.fixture(scope="module")
def fx():
    z, meta = LF.load()
    return z, meta, LF.cases(z, meta)


@pytest.mark.parametrize("mode", ["standard", "fl_epoch_plus_dlbcl", "probabilistic"])
def test_host_draws_reproduce_reference_loader(fx, mode):
    z, meta, vols = fx
    aug = meta[f"trainer/{mode}/config"]["augmentation"]
    pre = f"loader/{mode}/"
    names = meta[pre + "loaders"]
    dss = {nm: host_dataset(LF.dataset_state(z, meta, pre + nm + "/"), vols, aug) for nm in names}
    LF.set_rng(z, pre + "rng_before/")
    for nm in names:
        loader = LP.DevicePatchLoader(dss[nm], meta["batch"])
        assert len(loader) == meta[pre + nm + "/len"]
        sums = []
        for b, (x, t) in enumerate(loader):
            x, t = x.numpy(), t.numpy()
            sums.append(LF.batch_sums(x, t))
            if b < meta["k_batches"]:
                xr, tr = z[f"{pre}{nm}/x{b}"], z[f"{pre}{nm}/t{b}"]
                assert x.shape == xr.shape, (mode, nm, b, x.shape, xr.shape)
                assert np.abs(x - xr).max() <= 1e-6, (mode, nm, b, np.abs(x - xr).max())
                assert (t != tr).sum() <= 1e-4 * t.size, (mode, nm, b)
        ref = z[pre + nm + "/sums"]
        assert len(sums) == len(ref)
        np.testing.assert_allclose(np.array(sums), ref, rtol=1e-6, atol=1e-3)
    assert all(LF.rng_matches(z, pre + "rng_after/")), (mode, LF.rng_matches(z, pre + "rng_after/"))
    if pre + "counts" in meta:
        ds = dss[names[0]]
        assert ds.get_sample_counts() == meta[pre + "counts"]
