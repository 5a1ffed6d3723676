"""Data-parallel training entry for the reference Trainer on the MI355X hot path.

The reference trains on one device (scripts/train.py:26-59 -> Trainer(config).train()).  This
entry runs the same Trainer with l3u_plugin.install(fast_step=True) (graph-replayed TrainStep
loops, light_unet/fast_trainer.py), one process per GPU:

    PYTHONPATH=<reference repo>:<this dir> python -m torch.distributed.run --nnodes 1 \\
        --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29500 \\
        light-3d-unet-front_amd/l3u_train.py --config configs/unet_fl70.yaml

Every rank builds the Trainer from the same config (same seed -> the same initial weights, and
FastLoop broadcasts rank 0's anyway) and draws its own batches: the reference's PatchDataset
samples patches at random regardless of the index (patch_dataset.py:114-124), so seeding the
data pipeline per rank (experiment.seed + rank) is the sharding; the global batch is
batch_size * world.  The step's exchange (exchange.py) keeps the global-batch FocalTversky
(`--ftl-mode exact`, default) or plain DDP averaging (`local`).  Rank 0 keeps the configured
output directories; rank r > 0 writes its logs / TensorBoard under `<dir>_rank<r>`.
Validation (sliding-window inference + lesion metrics, trainer.py:349-458) runs on rank 0 only;
its result is broadcast, so every rank takes the same model-selection, scheduler and
early-stopping decisions (trainer.py:505-541) and the ranks' collectives stay in step.  Only
rank 0 writes checkpoints (the weights are identical on every rank after each step's gradient
all-reduce).  Unlike scripts/train.py:55 the config file is never rewritten.
"""
import argparse
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))


# how long ranks > 0 may wait for rank 0's validation (sliding-window inference + lesion metrics
# over the whole validation split, trainer.py:349-458)
VALIDATION_TIMEOUT_S = float(os.environ.get("L3U_VALIDATION_TIMEOUT_S", str(6 * 3600)))


def share_validation(trainer, rank, dist, timeout_s=None):
    """Trainer.validate on rank 0 only, its (val_loss, metrics) broadcast to every rank; no
    checkpoint files from ranks > 0.  The broadcast goes over a gloo side group with its own long
    timeout (VALIDATION_TIMEOUT_S): ranks > 0 wait there, on the host, for the whole of rank 0's
    validation, never inside an NCCL collective that the RCCL watchdog would abort (its default
    timeout is 10 minutes)."""
    import datetime
    ref_validate = trainer.validate
    side = dist.new_group(backend="gloo", timeout=datetime.timedelta(
        seconds=VALIDATION_TIMEOUT_S if timeout_s is None else timeout_s))

    def validate(epoch):
        out = [ref_validate(epoch) if rank == 0 else None]
        dist.broadcast_object_list(out, src=0, group=side)
        return out[0]
    trainer.validate = validate
    if rank > 0:
        trainer.save_checkpoint = lambda epoch, is_best=False: None


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", required=True)
    ap.add_argument("--data_dir", default=None)
    ap.add_argument("--splits_dir", default=None)
    ap.add_argument("--ftl-mode", default="exact", choices=["exact", "local"])
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--device-patches", action="store_true",
                    help="cut and augment training patches on the device (l3u_amd.patches; "
                         "num_workers = 0 draw semantics, per-rank RNG streams)")
    a = ap.parse_args(argv)

    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        if a.backend == "nccl":   # RCCL over xGMI
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    if _HERE not in sys.path:
        sys.path.insert(0, _HERE)
    import l3u_plugin
    l3u_plugin.install(fast_step=True, device_patches=a.device_patches)
    from light_unet.core.config import ConfigManager
    from light_unet.core.trainer import Trainer

    config = ConfigManager.load(a.config)
    if a.data_dir:
        config["data_dir"] = a.data_dir
    if a.splits_dir:
        config["splits_dir"] = a.splits_dir
    if rank > 0:
        for k in ("log_dir", "tensorboard_dir", "checkpoint_dir"):
            if k in config.get("output", {}):
                config["output"][k] = f"{config['output'][k]}_rank{rank}"
    trainer = Trainer(config)
    trainer.l3u_ftl_mode = a.ftl_mode
    if world > 1:   # per-rank data streams (the model is broadcast from rank 0 by FastLoop)
        import random
        import numpy as np
        seed = int(config["experiment"]["seed"]) + rank
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
    if world > 1:
        share_validation(trainer, rank, dist)
    trainer.train()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
