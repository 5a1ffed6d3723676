"""Per-launch floor of dependent kernels on this GPU: eager stream vs hipGraph replay, for a
1-workgroup kernel (l3u_counter_add) and a 512-workgroup elementwise kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

dev = torch.device("cuda:0")
cnt = torch.zeros(1, dtype=torch.int32, device=dev)
x = torch.rand(4, 64, 1728, device=dev)
rec = torch.rand(4 * 64, 8, device=dev)
out = torch.empty_like(x)
K = 200


def tiny():
    nat.call("l3u_counter_add", cnt.data_ptr(), 1, nat.stream())


def elem():
    nat.call("l3u_norm_act_fwd", x.data_ptr(), 64 * 1728, rec.data_ptr(), None, x.data_ptr(),
             64 * 1728, None, None, 0, out.data_ptr(), 64 * 1728, 4, 64, 1728, nat.stream())


def mixed():
    tiny()
    elem()


def step_like():
    # the real step's first kernels in order: is the floor different inside the training graph?
    pass


for name, fn in (("counter_add 1x1", tiny), ("norm_act 12^3 x64ch", elem), ("alternating", mixed)):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(K):
        fn()
    e1.record()
    torch.cuda.synchronize()
    eager = e0.elapsed_time(e1) / K * 1e3
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(K):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    graph = e0.elapsed_time(e1) / (5 * K) * 1e3
    print(f"{name:22s} eager {eager:6.2f} us/launch   graph {graph:6.2f} us/launch", flush=True)
