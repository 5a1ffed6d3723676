"""Does a kernel boundary cost more after a kernel that leaves much dirty data in L2?
Graph-replayed sequences: [big]xK, [big, tiny]xK, [tiny]xK; big = norm_act over 48^3 x 16ch x 4
(writes 28 MB), tiny = 1-workgroup counter increment."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

dev = torch.device("cuda:0")
cnt = torch.zeros(1, dtype=torch.int32, device=dev)
S = 48 ** 3
x = torch.rand(4, 16, S, device=dev)
rec = torch.rand(4 * 16, 8, device=dev)
out = torch.empty_like(x)
xs = torch.rand(4, 64, 1728, device=dev)
outs = torch.empty_like(xs)
recs = torch.rand(4 * 64, 8, device=dev)
K = 50


def tiny():
    nat.call("l3u_counter_add", cnt.data_ptr(), 1, nat.stream())


def big():
    nat.call("l3u_norm_act_fwd", x.data_ptr(), 16 * S, rec.data_ptr(), None, x.data_ptr(), 16 * S,
             None, None, 0, out.data_ptr(), 16 * S, 4, 16, S, nat.stream())


def small():
    nat.call("l3u_norm_act_fwd", xs.data_ptr(), 64 * 1728, recs.data_ptr(), None, xs.data_ptr(),
             64 * 1728, None, None, 0, outs.data_ptr(), 64 * 1728, 4, 64, 1728, nat.stream())


def timed(seq):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for f in seq:
            f()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(K):
            for f in seq:
                f()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * K) * 1e3


tb, tt, ts = timed([big]), timed([tiny]), timed([small])
tbt, tbs, tst = timed([big, tiny]), timed([big, small]), timed([small, tiny])
print(f"big {tb:.2f}  tiny {tt:.2f}  small {ts:.2f} us", flush=True)
print(f"big+tiny {tbt:.2f} (tiny after big costs {tbt - tb:.2f})  big+small {tbs:.2f} "
      f"(small after big costs {tbs - tb:.2f})  small+tiny {tst:.2f}", flush=True)
