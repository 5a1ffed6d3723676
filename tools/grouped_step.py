"""Graph-replayed train steps of the grouped (use_depthwise_separable=False) model, for a
rocprofv3 kernel trace of that variant (bench.py's grouped_1gpu leg, same workload):
    rocprofv3 --kernel-trace --stats -d OUT -o run -- python tools/grouped_step.py [steps]"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "light-3d-unet-front_amd"))
import torch  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = Lightweight3DUNet(dropout_p=0.1, use_depthwise_separable=False).to(dev).train()
    step = TrainStep(model, {"alpha": 0.7, "beta": 0.3, "gamma": 0.75}, lr=1e-4, weight_decay=1e-5,
                     distributed=False)
    rng = np.random.default_rng(42)
    bs, size = 4, 48
    xs = torch.from_numpy(rng.random((bs, 1, size, size, size), dtype=np.float32)).to(dev)
    ts = torch.from_numpy((rng.random((bs, 1, size, size, size)) > 0.97).astype(np.float32)).to(dev)
    step.capture(xs, ts, warmup=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        loss = step.replay()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"grouped step {1000 * dt / steps:.4f} ms, loss {float(loss.item()):.6f}")


if __name__ == "__main__":
    main()
