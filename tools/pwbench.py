"""Microbenchmark of the 1x1-conv backward at the model's shapes: the fused l3u_pw_bwd against
the unfused sequence (l3u_in_bwd_apply +) l3u_pw_fwd (data) + l3u_pw_bwd_weight.  Each variant
is captured as a graph of `iters` back-to-back launches and timed with events.

    python tools/pwbench.py [--iters 40]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))

import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

# (N, J, K, edge, in_prologue, accumulate, role)
SHAPES = [
    (4, 16, 16, 48, False, False, "init conv2 / up3 conv2"),
    (4, 16, 1, 48, True, False, "init conv1"),
    (4, 16, 1, 48, False, True, "init shortcut"),
    (4, 16, 32, 48, True, False, "up3 conv1"),
    (4, 16, 32, 48, False, True, "up3 shortcut"),
    (4, 32, 32, 24, False, False, "down1/up2 conv2"),
    (4, 32, 16, 24, True, False, "down1 conv1"),
    (4, 32, 16, 24, False, True, "down1 shortcut"),
    (4, 32, 64, 24, True, False, "up2 conv1"),
    (4, 32, 64, 24, False, True, "up2 shortcut"),
    (4, 64, 64, 12, False, False, "down2/up1 conv2"),
    (4, 64, 32, 12, True, False, "down2 conv1"),
    (4, 64, 32, 12, False, True, "down2 shortcut"),
    (4, 64, 128, 12, True, False, "up1 conv1"),
    (4, 64, 128, 12, False, True, "up1 shortcut"),
    (4, 128, 128, 6, False, False, "down3/bottleneck conv2"),
    (4, 128, 64, 6, True, False, "down3 conv1"),
    (4, 128, 64, 6, False, True, "down3 shortcut"),
    (4, 128, 128, 6, True, False, "bottleneck conv1"),
]


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
    for _ in range(5):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / (5 * iters) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--convt-only", action="store_true")
    ap.add_argument("--scale", action="store_true",
                    help="the fused backward at N = 1, 2, 4, 8 for the big shapes (bandwidth vs "
                         "latency scaling)")
    a = ap.parse_args()
    if a.scale:
        global SHAPES
        SHAPES = [(n, J, K, L, pro, acc, role) for (J, K, L, pro, acc, role) in
                  [(16, 32, 48, True, False, "up3 conv1"), (16, 32, 48, False, True, "up3 shortcut"),
                   (16, 16, 48, False, False, "up3 conv2"), (32, 64, 24, True, False, "up2 conv1"),
                   (32, 32, 24, False, False, "up2 conv2")] for n in (1, 2, 4, 8)]
    if a.convt_only:
        convt(a.iters)
        return
    dev = torch.device("cuda:0")
    tag = os.path.basename(os.environ.get("L3U_LIB", "default"))
    for (N, J, K, L, pro, acc, role) in SHAPES:
        S = L ** 3
        dy = torch.randn(N, J, S, device=dev)
        y = torch.randn(N, J, S, device=dev)
        x = torch.randn(N, K, S, device=dev)
        w = torch.randn(J, K, device=dev)
        dx = torch.zeros(N, K, S, device=dev)
        tmp = torch.empty(N, J, S, device=dev)
        rec = torch.rand(N * J, 8, device=dev)
        npart = 8
        ip = torch.rand(J * N * npart * 2, dtype=torch.float64, device=dev)
        P = max(nat.query("l3u_pw_bwd_weight_nparts", N, S), nat.query("l3u_pw_bwd_nparts", N, J, K, S))
        part = torch.empty(P * J * K, device=dev)

        def fused():
            st = torch.cuda.current_stream().cuda_stream
            pa = (y.data_ptr(), J * S, rec.data_ptr(), ip.data_ptr(), npart) if pro else (None, 0, None, None, 0)
            nat.call("l3u_pw_bwd", dy.data_ptr(), J * S, *pa, x.data_ptr(), K * S, w.data_ptr(),
                     dx.data_ptr(), K * S, int(acc), part.data_ptr(), N, J, K, S, st)

        def unfused():
            st = torch.cuda.current_stream().cuda_stream
            src = dy
            if pro:
                nat.call("l3u_in_bwd_apply", dy.data_ptr(), J * S, y.data_ptr(), J * S, rec.data_ptr(),
                         ip.data_ptr(), npart, tmp.data_ptr(), J * S, N, J, S, st)
                src = tmp
            nat.call("l3u_pw_fwd", src.data_ptr(), J * S, w.data_ptr(), 1, None, dx.data_ptr(), K * S,
                     int(acc), None, N, J, K, S, st)
            nat.call("l3u_pw_bwd_weight", src.data_ptr(), J * S, x.data_ptr(), K * S, part.data_ptr(),
                     N, J, K, S, st)

        nb = 4 * N * S * (J * (2 if pro else 1) + K + K * (2 if acc else 1))
        tf = graph_time(fused, a.iters)
        tu = graph_time(unfused, a.iters) if not a.scale else float("nan")
        print(f"{tag:12s} N{N} J{J:<3d} K{K:<3d} {L}^3 pro={int(pro)} acc={int(acc)} {role:24s} fused "
              f"{tf:7.2f} us ({nb / tf / 1e3:5.0f} GB/s)  unfused {tu:7.2f} us", flush=True)
    if not a.scale:
        convt(a.iters)


def convt(iters):
    dev = torch.device("cuda:0")
    for (N, Ci, Co, L) in [(4, 32, 16, 24), (4, 64, 32, 12), (4, 128, 64, 6), (4, 64, 32, 32),
                           (4, 128, 64, 16)]:
        Si = L ** 3
        dcat = torch.randn(N, 2 * Co, 8 * Si, device=dev)
        x = torch.randn(N, Ci, Si, device=dev)
        w = torch.randn(Ci, Co * 8, device=dev)
        dx = torch.empty(N, Ci, Si, device=dev)
        P = nat.query("l3u_convt_bwd_fused_nparts", N, Ci, Co, L, L, L)
        if P == 0:
            print(f"convT bwd Ci{Ci} Co{Co} {L}^3: one-launch form not offered")
            continue
        wp, bp = torch.empty(P * Ci * Co * 8, device=dev), torch.empty(P * Co, device=dev)
        P2 = nat.query("l3u_pw_bwd_weight_nparts", N, Si)
        wp2 = torch.empty(P2 * Ci * Co * 8, device=dev)
        bp2 = torch.empty(P2 * Co, device=dev)

        def fused():
            nat.call("l3u_convt_bwd_fused", dcat.data_ptr(), 2 * Co * 8 * Si, x.data_ptr(), Ci * Si,
                     w.data_ptr(), dx.data_ptr(), Ci * Si, wp.data_ptr(), bp.data_ptr(), N, Ci, Co,
                     L, L, L, torch.cuda.current_stream().cuda_stream)

        def unfused():
            nat.call("l3u_convt_bwd", dcat.data_ptr(), 2 * Co * 8 * Si, x.data_ptr(), Ci * Si,
                     w.data_ptr(), dx.data_ptr(), Ci * Si, wp2.data_ptr(), bp2.data_ptr(), N, Ci, Co,
                     L, L, L, torch.cuda.current_stream().cuda_stream)

        tf, tu = graph_time(fused, iters), graph_time(unfused, iters)
        byt = 4 * N * Si * (8 * Co + 2 * Ci)   # dY + X + dX (algorithmic)
        print(f"convT bwd Ci{Ci} Co{Co} {L}^3: one launch {tf:7.2f} us ({byt / tf / 1e3:6.0f} GB/s, "
              f"{P} partials)  three launches {tu:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
