"""Is the graph-replayed training step GPU-bound or submission-bound?  Reports the CPU time of
step.replay() calls, the GPU time of one isolated replay (events, after a sync) and the
pipelined per-step time."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402
from light_unet.train_step import TrainStep  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(42)
model = Lightweight3DUNet().to(dev).train()
x = torch.rand(4, 1, 48, 48, 48, device=dev)
t = (torch.rand(4, 1, 48, 48, 48, device=dev) > 0.97).float()
step = TrainStep(model)
step.capture(x, t)
for _ in range(5):
    step.replay()
torch.cuda.synchronize()
# isolated GPU time of one replay
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
iso = []
for _ in range(10):
    torch.cuda.synchronize()
    e0.record()
    step.replay()
    e1.record()
    torch.cuda.synchronize()
    iso.append(e0.elapsed_time(e1))
# CPU cost of submitting replays (no sync in between)
cpu = []
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    a = time.perf_counter()
    step.replay()
    cpu.append(time.perf_counter() - a)
torch.cuda.synchronize()
wall = (time.perf_counter() - t0) / 50
print(f"isolated replay GPU {sorted(iso)[5]:.3f} ms | replay() CPU {1e3 * sorted(cpu)[25]:.3f} ms "
      f"| pipelined {1e3 * wall:.3f} ms/step", flush=True)

# --- cost of the 12^3 / 6^3 levels inside the step graph: re-capture with those launches
# skipped (results meaningless; timing only)
from light_unet import _native as nat  # noqa: E402

orig = nat.call
small_sizes = {6, 12, 216, 1728, 3 * 216, 8 * 216, 8 * 1728}
skipped = [0]


def call(name, *args):
    ints = [a for a in args[:-1] if isinstance(a, int) and 0 <= a < (1 << 31)]   # no ptrs/stream
    tail = ints[-5:]
    if any(v in small_sizes for v in tail) and not any(v >= 13824 for v in tail):
        skipped[0] += 1
        return 0
    return orig(name, *args)


nat.call = call
step2 = TrainStep(model)
step2.capture(x, t)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(50):
    step2.replay()
torch.cuda.synchronize()
wall2 = (time.perf_counter() - t0) / 50
print(f"without 12^3/6^3 launches ({skipped[0] // 3} per step): {1e3 * wall2:.3f} ms/step", flush=True)
