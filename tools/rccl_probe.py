"""The data-parallel step on a real RCCL
("nccl") process group of ONE rank on the one-GPU box, before any 8-GPU run.

  single    TrainStep(distributed=False): one hipGraph, the fused gradient reduction + AdamW;
  segmented TrainStep(force_exchange=True): the world > 1 protocol -- fp64 FocalTversky sums
            all-reduced between the forward and the loss, the flat gradient all-reduced after the
            backward, the separate update launch; three graph segments with eager RCCL collectives;
  captured  the same with capture_collectives=True: the two RCCL all-reduces inside the graph.

Every variant starts from the same weights and replays the same batches; the worker writes the
parameters / losses after each step, and the per-step times of the three graph forms (the
exchange's cost on one GPU) to <out>/rccl.npz and <out>/rccl.json.  Run by
tests/test_rccl_gpu.py and by bench.py's `exchange` leg as a plain python subprocess (so the
caller never holds a process group); it creates its own TCP rendezvous on 127.0.0.1.

    python tools/rccl_probe.py <out dir> <port>"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "light-3d-unet-front_amd")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

SIZE = int(os.environ.get("RCCL_SIZE", "48"))
STEPS = 3


def batches(n, size=SIZE):
    rng = np.random.default_rng(11)
    out = []
    for _ in range(n):
        x = rng.random((4, 1, size, size, size), dtype=np.float32)
        t = (rng.random((4, 1, size, size, size)) > 0.97).astype(np.float32)
        out.append((x, t))
    return out


def main():
    out, port = sys.argv[1], int(sys.argv[2])
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=dev)
    assert dist.get_backend() == "nccl"
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    bt = batches(STEPS)
    dx = [torch.from_numpy(x).to(dev) for x, _ in bt]
    dt = [torch.from_numpy(t).to(dev) for _, t in bt]
    res, times = {}, {}
    for name, kw in (("single", dict(distributed=False)),
                     ("segmented", dict(force_exchange=True, capture_collectives=False)),
                     ("captured", dict(force_exchange=True, capture_collectives=True))):
        torch.manual_seed(42)
        m = Lightweight3DUNet(dropout_p=0.1).to(dev).train()
        ts = TrainStep(m, {"alpha": 0.7, "beta": 0.3, "gamma": 0.75}, lr=1e-4, weight_decay=1e-5,
                       **kw)
        assert ts.exchange == (name != "single")
        xs, tsb = dx[0].clone(), dt[0].clone()
        ts.capture(xs, tsb)
        for i in range(STEPS):
            xs.copy_(dx[i])
            tsb.copy_(dt[i])
            loss = ts.replay()
            torch.cuda.synchronize()
            res[f"{name}_loss{i}"] = np.float64(loss.item())
            res[f"{name}_p{i}"] = ts.flat.cpu().numpy().copy()
        # per-step time of this graph form (same inputs every replay)
        for _ in range(5):
            ts.replay()
        torch.cuda.synchronize()
        best = []
        for _ in range(3):
            t0 = time.perf_counter()
            for _ in range(20):
                ts.replay()
            torch.cuda.synchronize()
            best.append((time.perf_counter() - t0) / 20 * 1e3)
        times[name] = min(best)
        del ts, m
        torch.cuda.synchronize()
    np.savez(os.path.join(out, "rccl.npz"), **res)
    rec = {"backend": dist.get_backend(), "world": dist.get_world_size(), "size": SIZE,
           "ms_per_step": times,
           "exchange_us": {k: round(1000 * (times[k] - times["single"]), 1)
                           for k in ("segmented", "captured")}}
    with open(os.path.join(out, "rccl.json"), "w") as f:
        json.dump(rec, f)
    print(json.dumps(rec), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
