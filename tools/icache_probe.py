"""Where does a small-level launch's time go when it follows a streaming launch?  Three graphs of
the same 6^3 IN-on-load depthwise forward (l3u_dw3_fwd with an l3u_norm_src: dwv_fwd XF, the
bottleneck's conv2.depthwise shape [4, 128, 6^3]) are replayed under a rocprofv3 kernel trace:

  A  thrash (a 512 MiB copy: caches cold), then the probe call           -> code and data cold
  B  the probe call twice                                                 -> code and data warm
  C  thrash, the same kernel on ANOTHER buffer set (code warm), then the probe call -> data cold

The probe call's duration in A - C is the price of fetching the kernel's code after a streaming
launch; C - B the price of its cold data.  (tools/steplist-style summary printed by
tools/icache_summary.py from the trace.)

    rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/icache_probe.py [xf]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

dev = torch.device("cuda:0")
XF = (sys.argv[1] if len(sys.argv) > 1 else "1") == "1"
N, C, D = 4, 128, 6
S = D ** 3
st = nat.stream()


def bufs():
    nsb = 4
    x = torch.rand(N, C, S, device=dev)
    part = torch.empty(N, C, nsb, 3, device=dev)
    part[..., 0] = S / nsb
    part[..., 1] = torch.rand(N, C, nsb, device=dev)
    part[..., 2] = torch.rand(N, C, nsb, device=dev)
    gb = torch.rand(2, C, device=dev)
    rec = torch.empty(N, C, 8, device=dev)
    src = nat.NormSrc(part.data_ptr(), nsb, 3, gb[0].data_ptr(), gb[1].data_ptr(), 0.0, 0x5EED, None,
                      rec.data_ptr(), None)
    y = torch.empty(N, C, S, device=dev)
    w = torch.rand(C, 27, device=dev)
    return dict(x=x, part=part, gb=gb, rec=rec, src=src, y=y, w=w)


P, Q = bufs(), bufs()
big_a = torch.empty(128 << 20, device=dev)   # 512 MiB
big_b = torch.empty_like(big_a)


def call(b):
    nat.call("l3u_dw3_fwd", b["x"].data_ptr(), C * S, b["w"].data_ptr(), None,
             nat.norm_src_ptr(b["src"]) if XF else None, b["y"].data_ptr(), C * S, N, C, D, D, D,
             nat.stream())


def thrash():
    big_b.copy_(big_a)


def graph(fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        fn()
    return g


def pat_a():
    for _ in range(4):
        thrash()
        call(P)


def pat_b():
    for _ in range(4):
        call(P)
        call(P)


def pat_c():
    for _ in range(4):
        thrash()
        call(Q)
        call(P)


for name, fn in (("A", pat_a), ("B", pat_b), ("C", pat_c)):
    g = graph(fn)
    torch.cuda.synchronize()
    for _ in range(10):
        g.replay()
    torch.cuda.synchronize()
    print("pattern", name, "done", flush=True)
