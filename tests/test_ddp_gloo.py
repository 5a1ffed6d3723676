"""World-size-2 data-parallel protocol on CPU (gloo): the exchange functions the GPU TrainStep
uses (light_unet.exchange) reproduce the single-process global-batch step.

Each rank runs the fp64 oracle network on its shard of a batch of 4 (2 per rank), exchanges the
FocalTversky sums, forms dL/dp from the GLOBAL sums, backpropagates, and exchanges the flat
gradient.  In exact mode the result must equal autograd of the reference loss over the whole
batch on one process (losses.py:40-46 sums over every voxel of the batch); in local mode it must
equal the mean of the per-rank losses' gradients (plain DDP).  The oracle here is the checker;
the exchange code under test is the product's.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "light-3d-unet-front_amd")
ENC = (4, 8, 16, 32)
SIZE = 16
BATCH = 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem():
    from oracle.unet_oracle import param_names
    g = torch.Generator().manual_seed(7)
    sd = {}
    for name, shape in param_names(ENC):
        if name.endswith(("norm1.weight", "norm2.weight", "shortcut.1.weight")):   # IN gamma
            sd[name] = 1.0 + 0.1 * torch.randn(shape, generator=g, dtype=torch.float64)
        else:
            fan = max(1, int(torch.tensor(shape[1:]).prod()))
            sd[name] = torch.randn(shape, generator=g, dtype=torch.float64) / fan ** 0.5
    x = torch.rand((BATCH, 1, SIZE, SIZE, SIZE), generator=g, dtype=torch.float64)
    t = (torch.rand((BATCH, 1, SIZE, SIZE, SIZE), generator=g) > 0.9).double()
    return sd, x, t


def _flat_grad(sd, pred, dp):
    names = list(sd)
    grads = torch.autograd.grad(pred, [sd[n] for n in names], grad_outputs=dp)
    return torch.cat([g.reshape(-1) for g in grads])


def _reference(mode, world):
    """Single process: exact = gradient of the global-batch loss; local = mean of per-shard
    loss gradients."""
    from oracle.unet_oracle import focal_tversky, unet_forward
    sd, x, t = _problem()
    for v in sd.values():
        v.requires_grad_(True)
    if mode == "exact":
        loss = focal_tversky(unet_forward(sd, x), t)
    else:
        per = BATCH // world
        loss = sum(focal_tversky(unet_forward(sd, x[r * per:(r + 1) * per]), t[r * per:(r + 1) * per])
                   for r in range(world)) / world
    grads = torch.autograd.grad(loss, list(sd.values()))
    return torch.cat([g.reshape(-1) for g in grads]), loss.detach()


def _rank(rank, world, port, mode, outdir):
    for p in (ROOT, PKG):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch.distributed as dist
    from light_unet.exchange import exchange_ftl_sums, exchange_grads
    from oracle.unet_oracle import ftl_grad_closed_form, ftl_sums, unet_forward
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    try:
        sd, x, t = _problem()
        for v in sd.values():
            v.requires_grad_(True)
        per = BATCH // world
        xs, ts = x[rank * per:(rank + 1) * per], t[rank * per:(rank + 1) * per]
        pred = unet_forward(sd, xs)
        sums = ftl_sums(pred.detach(), ts)
        local = sums.clone()
        exchange_ftl_sums(sums, mode)
        dp = ftl_grad_closed_form(pred.detach(), ts, sums=sums)
        g = _flat_grad(sd, pred, dp)
        exchange_grads(g, mode)
        torch.save({"g": g, "sums": sums, "local": local}, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["exact", "local"])
def test_two_rank_step_matches_single_process(mode, tmp_path):
    world = 2
    mp.spawn(_rank, args=(world, _free_port(), mode, str(tmp_path)), nprocs=world, join=True)
    outs = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    ref, _ = _reference(mode, world)
    # every rank ends with the same gradient
    assert torch.equal(outs[0]["g"], outs[1]["g"])
    rel = (outs[0]["g"] - ref).norm() / ref.norm()
    assert rel < 1e-10, rel
    if mode == "exact":
        tot = outs[0]["local"] + outs[1]["local"]
        assert torch.allclose(outs[0]["sums"], tot, rtol=1e-12, atol=0)
    else:
        assert torch.equal(outs[0]["sums"], outs[0]["local"])


def test_local_and_exact_differ():
    """The exact protocol is not plain DDP: on a lesion-sparse batch the two gradients differ
    (SURVEY §8e measured ~0.3% at bs 4x2); guards against the modes silently collapsing."""
    ge, _ = _reference("exact", 2)
    gl, _ = _reference("local", 2)
    assert (ge - gl).norm() / ge.norm() > 1e-4


def test_mode_validation():
    from light_unet.exchange import check_mode
    with pytest.raises(ValueError):
        check_mode("sum")


def _share_validation_worker(rank, world, port, q, slow_s=0.0):
    import datetime
    import sys as _s
    import time as _t
    _s.path.insert(0, PKG)
    import torch.distributed as dist
    import l3u_train
    # the main group's collectives time out after 3 s: a validation longer than that must not
    # reach them (the RCCL watchdog stands in here)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world, timeout=datetime.timedelta(seconds=3))

    class T:
        calls = 0
        saved = []

        def validate(self, epoch):
            T.calls += 1
            _t.sleep(slow_s)
            return 0.0, {"best_recall": 0.5 + epoch, "rank": rank}

        def save_checkpoint(self, epoch, is_best=False):
            T.saved.append(epoch)
    t = T()
    l3u_train.share_validation(t, rank, dist)
    res = [t.validate(e) for e in range(2)]
    t.save_checkpoint(0, True)
    q.put((rank, T.calls, res, list(T.saved)))
    dist.destroy_process_group()


def test_validation_on_rank0_broadcast():
    """l3u_train: Trainer.validate runs on rank 0 only and every rank receives its result (same
    scheduler / early-stopping decisions); ranks > 0 write no checkpoints.  Rank 0's validation
    takes 4 s, longer than the main group's 3 s collective timeout: rank 1 waits on the side
    group, so nothing times out."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_share_validation_worker, args=(r, 2, port, q, 4.0)) for r in range(2)]
    for p in ps:
        p.start()
    got = sorted(q.get(timeout=60) for _ in ps)
    for p in ps:
        p.join(30)
    assert got[0][1] == 2 and got[1][1] == 0
    assert got[0][2] == got[1][2] == [(0.0, {"best_recall": 0.5, "rank": 0}),
                                      (0.0, {"best_recall": 1.5, "rank": 0})]
    assert got[0][3] == [0] and got[1][3] == []
