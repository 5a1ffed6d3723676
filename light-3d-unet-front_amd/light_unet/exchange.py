"""Data-parallel exchange protocol of the training step.

The reference trains on one device; its loss (losses.py:40-46) sums tp/fp/fn over ALL voxels
of the batch.  Sharding the batch over ranks keeps that meaning only if the three sums are
combined before the loss is formed, so the step has two exchange points:

  exact (default)  all_reduce(SUM) of the 3 FocalTversky sums after the forward, then
                   all_reduce(SUM) of the flat gradient: the global loss is one function of
                   every rank's voxels, and its gradient is the sum of the per-rank pieces;
  local            no sums exchange (each rank's own loss), gradients averaged (plain DDP).

Both collectives act on ONE flat buffer each (24 B of fp64 sums; the 0.87 MB flat gradient),
RCCL over xGMI on the GPU ("nccl" backend), gloo in the CPU tests.  The functions are backend
agnostic so the protocol itself is tested on CPU (tests/test_ddp_gloo.py).
"""
import torch.distributed as dist

MODES = ("exact", "local")


def check_mode(mode):
    if mode not in MODES:
        raise ValueError("ftl_mode must be 'exact' or 'local'")
    return mode


def world_size(group=None):
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group)
    return 1


def exchange_ftl_sums(sums, mode, group=None, force=False):
    """In place: the (tp, fp, fn) sums of this rank's shard -> the global-batch sums (exact).
    force: issue the collective even in a one-rank group (tests the RCCL path on one GPU)."""
    if (world_size(group) > 1 or force) and mode == "exact":
        dist.all_reduce(sums, op=dist.ReduceOp.SUM, group=group)
    return sums


def exchange_grads(gflat, mode, group=None, force=False):
    """In place: this rank's flat gradient -> the gradient of the global objective."""
    w = world_size(group)
    if w > 1 or force:
        if mode == "local":
            dist.all_reduce(gflat, op=dist.ReduceOp.SUM, group=group)
            gflat.div_(w)
        else:
            dist.all_reduce(gflat, op=dist.ReduceOp.SUM, group=group)
    return gflat
