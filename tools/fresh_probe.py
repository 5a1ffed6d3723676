"""How long does a small-level launch take to read data its predecessor just wrote?  Graph-replayed
pairs at the bottleneck level ([4, 128, 6^3]): the producer l3u_pw_fwd (128 -> 128, with the IN
statistics partials) writes y; the consumer l3u_dw3_fwd reads y (plain, and with the InstanceNorm
record finalized from those partials: the step's conv2.depthwise).  Patterns (consumer duration
classified by tools/fresh_summary.py from the rocprofv3 kernel trace):

  F  producer -> consumer                     the consumer reads fresh data
  O  producer -> other GEMM -> consumer       the data is one launch older
  W  consumer -> consumer                     warm (same inputs again)

Run it under variant libraries (e.g. L3U_ST_NT=1, non-temporal producer stores) to see whether
the producer's store policy changes the consumer's first-read latency.

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/fresh_probe.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

dev = torch.device("cuda:0")
N, C, D = 4, 128, 6
S = D ** 3
nsb = nat.query("l3u_pw_stat_nsb", C, C, S)
x = torch.rand(N, C, S, device=dev)
y = torch.empty(N, C, S, device=dev)
y2 = torch.empty(N, C, S, device=dev)
z = torch.empty(N, C, S, device=dev)
w = torch.rand(C, C, device=dev) / C ** 0.5
wd = torch.rand(C, 27, device=dev)
part = torch.empty(N * C * nsb * 3, device=dev)
part2 = torch.empty_like(part)
gb = torch.rand(2, C, device=dev)
rec = torch.empty(N, C, 8, device=dev)
src = nat.NormSrc(part.data_ptr(), nsb, 3, gb[0].data_ptr(), gb[1].data_ptr(), 0.0, 0x5EED, None,
                  rec.data_ptr(), None)
XF = (sys.argv[1] if len(sys.argv) > 1 else "1") == "1"


def prod(out, pt):
    nat.call("l3u_pw_fwd", x.data_ptr(), C * S, w.data_ptr(), 0, None, out.data_ptr(), C * S, 0,
             pt.data_ptr(), N, C, C, S, nat.stream())


def cons():
    nat.call("l3u_dw3_fwd", y.data_ptr(), C * S, wd.data_ptr(), None,
             nat.norm_src_ptr(src) if XF else None, z.data_ptr(), C * S, N, C, D, D, D, nat.stream())


def pat_f():
    for _ in range(8):
        prod(y, part)
        cons()


def pat_o():
    for _ in range(8):
        prod(y, part)
        prod(y2, part2)
        cons()


def pat_w():
    for _ in range(8):
        cons()
        cons()


for name, fn in (("F", pat_f), ("O", pat_o), ("W", pat_w)):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    print("pattern", name, "done", flush=True)
