"""Per-launch cost of the small-level (6^3 / 12^3) C-ABI calls in a replayed graph of K
back-to-back launches, each reading the previous launch's output (ping-pong buffers, as inside
the step): the warm steady-state cost of a launch, to set against its in-step duration.

    python tools/smallbench.py [K]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 40
dev = torch.device("cuda:0")
N = 4


def per_launch(step):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(3):
            step(i)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for i in range(K):
            step(i)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 20 / K * 1e6


def main():
    for L, C in ((6, 128), (12, 64), (24, 32)):
        S = L ** 3
        a = [torch.rand(N, C, S, device=dev) for _ in range(2)]
        w = torch.rand(C, C, device=dev) * 0.1
        wd = torch.rand(C, 27, device=dev) * 0.1
        nsb = nat.query("l3u_pw_stat_nsb", C, C, S)
        part = torch.empty(N * C * nsb * 3, device=dev)
        rec = torch.rand(N * C, 8, device=dev)
        rec[:, 1] = 1.0

        def pw(i):
            nat.call("l3u_pw_fwd", a[i % 2].data_ptr(), C * S, w.data_ptr(), 0, None,
                     a[1 - i % 2].data_ptr(), C * S, 0, part.data_ptr(), N, C, C, S, nat.stream())

        def dw(i):
            nat.call("l3u_dw3_fwd", a[i % 2].data_ptr(), C * S, wd.data_ptr(), None, None,
                     a[1 - i % 2].data_ptr(), C * S, N, C, L, L, L, nat.stream())

        def dwx(i):
            nat.call("l3u_dw3_fwd", a[i % 2].data_ptr(), C * S, wd.data_ptr(), rec.data_ptr(), None,
                     a[1 - i % 2].data_ptr(), C * S, N, C, L, L, L, nat.stream())

        gam = torch.ones(C, device=dev)
        bet = torch.zeros(C, device=dev)
        src = nat.NormSrc(part.data_ptr(), nsb, 3, gam.data_ptr(), bet.data_ptr(), 0.0, 1, None, None, None)

        def dws(i):   # IN record finalized in-kernel from GEMM partials
            nat.call("l3u_dw3_fwd", a[i % 2].data_ptr(), C * S, wd.data_ptr(), None,
                     nat.norm_src_ptr(src), a[1 - i % 2].data_ptr(), C * S, N, C, L, L, L, nat.stream())

        def tail(i):
            nat.call("l3u_norm_act_fwd", a[i % 2].data_ptr(), C * S, rec.data_ptr(), None,
                     a[i % 2].data_ptr(), C * S, None, None, 0, a[1 - i % 2].data_ptr(), C * S, N, C,
                     S, nat.stream())

        pw(0)
        torch.cuda.synchronize()
        for name, fn in (("pw_fwd+stats", pw), ("dw3_fwd", dw), ("dw3_fwd rec", dwx),
                         ("dw3_fwd src", dws), ("norm_act_fwd", tail)):
            print(f"[{N},{C},{L}^3] {name:14s} {per_launch(fn):6.2f} us per launch", flush=True)


if __name__ == "__main__":
    main()
