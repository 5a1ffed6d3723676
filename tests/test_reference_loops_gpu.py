"""GPU: the device training loaders and the graph-replayed Trainer loops against the REFERENCE's
own loaders and Trainer (tests/golden/loops.npz, made by tests/golden/make_loop_goldens.py from
light_unet/datasets/loader.py, patch_dataset.py and light_unet/core/trainer.py themselves):

  * DevicePatchDataset / DeviceMixedPatchDataset (light_unet/patches.py), built from the states
    the reference datasets were built with (cases, sampled locations) and started from the
    recorded RNG states, reproduce the reference epoch: the first batches elementwise (images
    1e-6, labels <= 1e-4 of the voxels: nearest-neighbour ties), a checksum of every batch, the
    numpy / python / torch RNG states after the epoch and the mixed dataset's domain counts;
  * light_unet.fast_trainer's train_epoch / _train_epoch_step_based (the loops l3u_plugin binds
    onto the reference Trainer, trainer.py:208-347), on the reference model's initial weights and
    those device loaders, record the reference's scalars -- same tags at the same global steps
    in the same order, per-step losses and Domain scalars, and the same returned average -- for
    two epochs in the standard, fl_epoch_plus_dlbcl and probabilistic modes; the weights after
    both epochs agree with the reference's to the AdamW step-noise bound.
The reference runs in fp32 on the CPU, this path in fp32 on the GPU: losses agree to 2e-4
relative (measured well below; fp32 summation order)."""
import types

import numpy as np
import pytest
import torch

import loops_fixture as LF

pytestmark = pytest.mark.gpu

MODES = ["standard", "fl_epoch_plus_dlbcl", "probabilistic"]


@pytest.fixture(scope="module")
def fx():
    z, meta = LF.load()
    return z, meta, LF.cases(z, meta)


def device_dataset(st, vols, aug):
    from light_unet import patches as LP
    if st["kind"] == "mixed":
        return LP.DeviceMixedPatchDataset(device_dataset(dict(st["fl"], kind="patch"), vols, aug),
                                          device_dataset(dict(st["dlbcl"], kind="patch"), vols, aug),
                                          st["fl_ratio"])
    return LP.DevicePatchDataset([vols[c] for c in st["case_ids"]], st["patch_size"],
                                 st["lesion_patch_ratio"], aug,
                                 locations=(st["lesion"], st["background"]))


@pytest.mark.parametrize("mode", MODES)
def test_device_loaders_match_reference_batches(cuda, fx, mode):
    from light_unet import patches as LP
    z, meta, vols = fx
    aug = meta[f"trainer/{mode}/config"]["augmentation"]
    pre = f"loader/{mode}/"
    names = meta[pre + "loaders"]
    dss = {nm: device_dataset(LF.dataset_state(z, meta, pre + nm + "/"), vols, aug) for nm in names}
    LF.set_rng(z, pre + "rng_before/")
    for nm in names:
        loader = LP.DevicePatchLoader(dss[nm], meta["batch"])
        assert len(loader) == meta[pre + nm + "/len"]
        sums = []
        for b, (x, t) in enumerate(loader):
            x, t = x.cpu().numpy(), t.cpu().numpy()
            sums.append(LF.batch_sums(x, t))
            if b < meta["k_batches"]:
                xr, tr = z[f"{pre}{nm}/x{b}"], z[f"{pre}{nm}/t{b}"]
                assert x.shape == xr.shape, (mode, nm, b, x.shape, xr.shape)
                assert np.abs(x - xr).max() <= 1e-6, (mode, nm, b, np.abs(x - xr).max())
                assert (t != tr).sum() <= 1e-4 * t.size, (mode, nm, b)
        np.testing.assert_allclose(np.array(sums), z[pre + nm + "/sums"], rtol=1e-6, atol=1e-3)
    assert all(LF.rng_matches(z, pre + "rng_after/")), LF.rng_matches(z, pre + "rng_after/")
    if pre + "counts" in meta:
        assert dss[names[0]].get_sample_counts() == meta[pre + "counts"]


class _Writer:
    def __init__(self):
        self.log = []

    def add_scalar(self, tag, value, step):
        self.log.append((str(tag), int(step), float(value)))


@pytest.mark.parametrize("mode", MODES)
def test_fast_trainer_matches_reference_trainer(cuda, fx, mode):
    from light_unet import fast_trainer as FT
    from light_unet import patches as LP
    from light_unet.models.losses import FocalTverskyLoss
    from light_unet.models.unet3d import Lightweight3DUNet
    z, meta, vols = fx
    pre = f"trainer/{mode}/"
    cfg = meta[pre + "config"]
    mc, tc = cfg["model"], cfg["training"]
    model = Lightweight3DUNet(in_channels=1, out_channels=mc["output_channels"],
                              start_channels=mc["start_channels"],
                              encoder_channels=mc["encoder_channels"],
                              use_depthwise_separable=mc["use_depthwise_separable"],
                              use_grouped=mc["use_grouped_conv"], groups=mc["groups"],
                              dropout_p=mc["dropout_p"] if mc["use_dropout"] else 0.0)
    init = {k: torch.from_numpy(z[pre + "init/" + k].copy()) for k in model.state_dict()}
    model.load_state_dict(init)
    model = model.to(cuda)
    t = types.SimpleNamespace()
    t.model, t.config, t.writer = model, cfg, _Writer()
    lc = cfg["loss"]
    t.criterion = FocalTverskyLoss(alpha=lc["alpha"], beta=lc["beta"], gamma=lc["gamma"])
    t.optimizer = torch.optim.AdamW(model.parameters(), lr=tc["learning_rate"],
                                    weight_decay=tc["weight_decay"])
    loaders = {nm: LP.DevicePatchLoader(device_dataset(LF.dataset_state(z, meta, pre + nm + "/"), vols,
                                                       cfg["augmentation"]), tc["batch_size"])
               for nm in meta[pre + "loaders"]}
    t.use_step_based_mixed = mode == "fl_epoch_plus_dlbcl"
    t.use_mixed_training = mode == "probabilistic"
    t.train_loader = loaders.get("train_loader")
    t.fl_loader, t.dlbcl_loader = loaders.get("fl_loader"), loaders.get("dlbcl_loader")
    t.train_dataset = t.train_loader.dataset if mode == "probabilistic" else None
    t.train_epoch = types.MethodType(FT.train_epoch, t)
    t._train_epoch_step_based = types.MethodType(FT.train_epoch_step_based, t)
    LF.set_rng(z, pre + "rng_before/")
    worst = 0.0
    nsteps = 0
    for epoch in (0, 1):
        t.writer.log.clear()
        ret = t.train_epoch(epoch)
        ref = [tuple(s) for s in meta[pre + f"epoch{epoch}/scalars"]]
        got = t.writer.log
        assert [(g[0], g[1]) for g in got] == [(r[0], r[1]) for r in ref], (mode, epoch)
        for (tag, step, v), (_, _, rv) in zip(got, ref):
            if tag.startswith("Domain/"):
                assert v == pytest.approx(rv, abs=1e-12), (tag, step, v, rv)
            else:
                worst = max(worst, abs(v - rv) / abs(rv))
                assert abs(v - rv) <= 2e-4 * abs(rv), (mode, epoch, tag, step, v, rv)
        assert abs(ret - meta[pre + f"epoch{epoch}/return"]) <= 2e-4 * abs(ret), (ret, meta[pre + f"epoch{epoch}/return"])
        nsteps += sum(1 for g in got if g[0] == "Loss/train_step")
    print(f"{mode}: {nsteps} steps, worst loss rel diff {worst:.2e}")
    assert all(LF.rng_matches(z, pre + "rng_after/")), LF.rng_matches(z, pre + "rng_after/")
    # weights after both epochs: AdamW moves each element by <= ~lr per step, so fp32 order
    # differences on near-zero gradients are bounded by lr * steps; the trajectory as a whole
    # agrees to 1e-2 of the distance travelled
    lr = tc["learning_rate"]
    num, den = 0.0, 0.0
    for k, v in model.state_dict().items():
        a = v.detach().cpu().double().numpy()
        r = z[pre + "final/" + k].astype(np.float64)
        assert np.abs(a - r).max() <= lr * nsteps, (k, np.abs(a - r).max())
        num += ((a - r) ** 2).sum()
        den += ((r - z[pre + "init/" + k].astype(np.float64)) ** 2).sum()
    assert num ** 0.5 <= 1e-2 * den ** 0.5, (num ** 0.5, den ** 0.5)
