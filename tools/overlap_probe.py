"""Probe: do the latency-bound small levels of one half-batch overlap the bandwidth-bound big
levels of another?  Times graph-replayed training steps of independent models on separate HIP
streams (free-running, optionally offset by a device sleep) against the one-stream bs-4 step.

    python tools/overlap_probe.py [iters]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "light-3d-unet-front_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402
from light_unet.train_step import TrainStep  # noqa: E402

dev = torch.device("cuda:0")
ITERS = int(sys.argv[1]) if len(sys.argv) > 1 else 40


def mk(bs, seed):
    torch.manual_seed(42)
    m = Lightweight3DUNet(dropout_p=0.1).to(dev).train()
    ts = TrainStep(m, {"alpha": 0.7, "beta": 0.3, "gamma": 0.75}, lr=1e-4, weight_decay=1e-5,
                   distributed=False)
    rng = np.random.default_rng(seed)
    x = torch.from_numpy(rng.random((bs, 1, 48, 48, 48), dtype=np.float32)).to(dev)
    t = torch.from_numpy((rng.random((bs, 1, 48, 48, 48)) > 0.97).astype(np.float32)).to(dev)
    ts.capture(x, t, warmup=2)
    return ts


def run(steps, offsets_us, iters=ITERS):
    streams = [torch.cuda.Stream() for _ in steps]
    for s in streams:
        s.wait_stream(torch.cuda.current_stream())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s, off in zip(streams, offsets_us):
        if off:
            with torch.cuda.stream(s):
                torch.cuda._sleep(int(off * 2100))   # ~cycles at the shader clock
    for i in range(iters):
        for ts, s in zip(steps, streams):
            with torch.cuda.stream(s):
                ts._graphs[0].replay()
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / iters


one = mk(4, 1)
for _ in range(2):
    base = run([one], [0])
print(f"bs4 one stream: {base:.4f} ms/step")
h = [mk(2, 2), mk(2, 3)]
print(f"bs2 one stream: {run(h[:1], [0]):.4f} ms/step")
for off in (0, 150, 300, 450):
    print(f"2 x bs2 streams, offset {off} us: {run(h, [0, off]):.4f} ms per pair")
q = [mk(1, 4 + i) for i in range(4)]
print(f"bs1 one stream: {run(q[:1], [0]):.4f} ms/step")
for off in (0, 150):
    print(f"4 x bs1 streams, offsets k*{off} us: {run(q, [k * off for k in range(4)]):.4f} ms per quad")
