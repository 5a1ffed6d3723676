"""Worker of tests/test_model_gpu.py::test_trainstep_data_parallel_two_ranks (not a test module).

Every rank runs the product TrainStep (light_unet/train_step.py) on its half of a bs-4 batch:
  A  exact mode, dropout 0: one eager step (flat gradient after the exchange, loss), then
     capture() (the 3-segment graph with eager collectives between segments) and one replay
     on the next batch (parameters after both steps);
  B  local mode, dropout 0: one eager step (the averaged flat gradient);
  C  dropout 0.1: the Dropout3d keep scales the forward drew for every (block, n, c).
Rank r saves its arrays to <out>/rank<r>.npz.  Launched by torch.distributed.run (gloo, all
ranks on cuda:0; RCCL on a node).  argv: <out> [encoder channels, e.g. 16,32,64,128] [f32 | bf16]
[volume edge]: the network (BASELINE config 5: 32,64,128,256), the activation storage (config 3:
bf16) and the patch size of the run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "light-3d-unet-front_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SIZE = 32


def batches(n_steps, size=SIZE):
    """The global bs-4 batches every process draws identically (seeded)."""
    rng = np.random.default_rng(7)
    out = []
    for _ in range(n_steps):
        x = rng.random((4, 1, size, size, size), dtype=np.float32)
        t = (rng.random((4, 1, size, size, size)) > 0.97).astype(np.float32)
        out.append((x, t))
    return out


def fresh_model(dev, dropout_p, enc=(16, 32, 64, 128)):
    from light_unet.models.unet3d import Lightweight3DUNet
    torch.manual_seed(42)
    return Lightweight3DUNet(encoder_channels=list(enc), dropout_p=dropout_p).to(dev).train()


def parse(argv):
    """(encoder channels, activation dtype, volume edge) from the worker's argv[2:]"""
    enc = tuple(int(c) for c in argv[0].split(",")) if len(argv) > 0 else (16, 32, 64, 128)
    dt = torch.bfloat16 if len(argv) > 1 and argv[1] == "bf16" else torch.float32
    size = int(argv[2]) if len(argv) > 2 else SIZE
    return enc, dt, size


def main():
    out = sys.argv[1]
    enc, adt, size = parse(sys.argv[2:])
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from light_unet.train_step import TrainStep
    per = 4 // world
    sl = slice(rank * per, (rank + 1) * per)
    bt = batches(2, size)
    dx = [torch.from_numpy(x[sl].copy()).to(dev) for x, _ in bt]
    dt = [torch.from_numpy(t[sl].copy()).to(dev) for _, t in bt]
    res = {}
    # A: exact mode, eager step then graph replay
    m = fresh_model(dev, 0.0, enc)
    ts = TrainStep(m, ftl_mode="exact", dtype=adt)
    loss = ts(dx[0], dt[0])
    torch.cuda.synchronize()
    res["A_loss1"] = np.float64(loss.item())
    res["A_g1"] = ts.gflat.cpu().numpy().copy()
    xs, tsb = dx[1].clone(), dt[1].clone()
    ts.capture(xs, tsb)
    res["A_p1"] = ts.flat.cpu().numpy().copy()      # capture() must not move the parameters
    loss = ts.replay()
    torch.cuda.synchronize()
    res["A_loss2"] = np.float64(loss.item())
    res["A_p2"] = ts.flat.cpu().numpy().copy()
    # B: local mode (plain DDP averaging)
    m = fresh_model(dev, 0.0, enc)
    ts = TrainStep(m, ftl_mode="local", dtype=adt)
    ts(dx[0], dt[0])
    torch.cuda.synchronize()
    res["B_g1"] = ts.gflat.cpu().numpy().copy()
    # C: Dropout3d keep scales drawn by this rank's forward
    m = fresh_model(dev, 0.1, enc)
    m.engine.set_act_dtype(adt)
    _, sv = m.engine.forward(m.flat_parameters(), dx[0], training=True, dropout_p=0.1,
                             counter=m._rng_counter, save=True)
    torch.cuda.synchronize()
    for i, pre in enumerate(m.engine.BLOCKS):
        res[f"C_keep{i}"] = sv["blk"][pre]["recs"][1][:, 4].cpu().numpy()   # [n * C + c]
    np.savez(os.path.join(out, f"rank{rank}.npz"), **res)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
