"""Practical memory ceilings at the depthwise shapes: torch copy (1 read + 1 write stream),
read-only sum, and a 3-stream elementwise (2 reads + 1 write), in GB/s of algorithmic bytes."""
import torch


def timeit(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


dev = torch.device("cuda:0")
for (N, C, L) in [(4, 32, 48), (4, 16, 48), (32, 32, 48)]:
    n = N * C * L ** 3
    a = torch.rand(n, device=dev)
    b = torch.rand(n, device=dev)
    c = torch.empty(n, device=dev)
    u = 4 * n
    for name, fn, nb in [("copy", lambda: c.copy_(a), 2 * u), ("sum", lambda: a.sum(), u),
                         ("add3", lambda: torch.add(a, b, out=c), 3 * u)]:
        us = timeit(fn)
        print(f"{name:5s} [{N},{C},{L}^3] {us:8.2f} us {nb / us / 1e3:7.0f} GB/s", flush=True)
