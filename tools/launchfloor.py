"""Floor cost of one tiny launch inside a replayed hipGraph (wall time / launches)."""
import time
import torch
dev = torch.device("cuda:0")
for n_el in (256, 65536, 1 << 20):
    a = torch.zeros(n_el, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        for _ in range(3):
            a.add_(1.0)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(200):
            a.add_(1.0)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        g.replay()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / 50 / 200 * 1e6
    print(f"{n_el} elems: {us:.2f} us per launch in a graph", flush=True)
