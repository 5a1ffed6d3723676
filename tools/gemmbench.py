"""Microbenchmark of the channel GEMM launches of the step at the model's shapes: l3u_pw_fwd
(with and without IN statistics), l3u_convt_fwd (scatter epilogue) and l3u_convt_bwd (gathered
data + weight gradient).  Each case is captured as a graph of `iters` back-to-back launches and
timed with events.  Library chosen with L3U_LIB (variant builds).

    python tools/gemmbench.py [--iters 40]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))

import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

# (N, K, Nout, edge, stats): pointwise forward
PW = [(4, 16, 16, 48, True), (4, 32, 32, 24, True), (4, 64, 64, 12, True), (4, 128, 128, 6, True),
      (4, 64, 128, 6, True), (4, 128, 64, 12, True), (4, 32, 64, 12, True)]
# (N, Ci, Co, low-res edge): ConvTranspose3d
CT = [(4, 128, 64, 6), (4, 64, 32, 12), (4, 32, 16, 24)]


def graph_time(fn, iters):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    tag = os.path.basename(os.environ.get("L3U_LIB", "default"))
    for (N, K, J, L, stats) in PW:
        S = L ** 3
        x = torch.rand(N, K, S, device=dev)
        w = torch.rand(J, K, device=dev)
        y = torch.empty(N, J, S, device=dev)
        nsb = nat.query("l3u_pw_stat_nsb", K, J, S)
        sp = torch.empty(N * J * nsb * 3, device=dev)

        def fn():
            nat.call("l3u_pw_fwd", x.data_ptr(), K * S, w.data_ptr(), 0, None, y.data_ptr(), J * S, 0,
                     sp.data_ptr() if stats else None, N, K, J, S, nat.stream())
        print(f"{tag:18s} pw_fwd  N{N} K{K:4d} J{J:4d} {L}^3  {graph_time(fn, a.iters):8.2f} us", flush=True)
    for (N, Ci, Co, L) in CT:
        S = L ** 3
        x = torch.rand(N, Ci, S, device=dev)
        w = torch.rand(Ci, Co, 2, 2, 2, device=dev)
        b = torch.rand(Co, device=dev)
        out = torch.empty(N, Co, 8 * S, device=dev)

        def fn():
            nat.call("l3u_convt_fwd", x.data_ptr(), Ci * S, w.data_ptr(), b.data_ptr(), out.data_ptr(),
                     Co * 8 * S, N, Ci, Co, L, L, L, nat.stream())
        print(f"{tag:18s} ct_fwd  N{N} Ci{Ci:4d} Co{Co:4d} {L}^3  {graph_time(fn, a.iters):8.2f} us", flush=True)
        dy = torch.rand(N, Co, 8 * S, device=dev)
        dx = torch.empty(N, Ci, S, device=dev)
        P = nat.query("l3u_pw_bwd_weight_nparts", N, S)
        wp = torch.empty(P * Ci * Co * 8, device=dev)
        bp = torch.empty(max(1, P) * Co * 8, device=dev)

        def fb():
            nat.call("l3u_convt_bwd", dy.data_ptr(), Co * 8 * S, x.data_ptr(), Ci * S, w.data_ptr(),
                     dx.data_ptr(), Ci * S, wp.data_ptr(), bp.data_ptr(), N, Ci, Co, L, L, L, nat.stream())
        print(f"{tag:18s} ct_bwd  N{N} Ci{Ci:4d} Co{Co:4d} {L}^3  {graph_time(fb, a.iters):8.2f} us", flush=True)


if __name__ == "__main__":
    main()
