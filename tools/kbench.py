"""Kernel microbenchmark through the C-ABI: average launch time and algorithmic GB/s of the
depthwise stencil kernels at the model's shapes.  Library chosen with L3U_LIB (variant builds).

    python tools/kbench.py [--iters 50] [--which bwd,fwd,bwd1,bwdacc]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))

import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

SHAPES = [tuple(int(v) for v in t.split(",")) for t in os.environ.get(
    "KB_SHAPES", "4,32,48 4,16,48 4,64,24 4,32,24 4,16,24 4,128,12 4,64,12").split()]


FLUSH = None


def timeit(fn, iters):
    if FLUSH is not None:   # cold: a 512 MiB write evicts the 256 MiB MALL before every call
        for _ in range(2):
            fn()
        tot = 0.0
        for _ in range(iters):
            FLUSH.add_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            tot += e0.elapsed_time(e1)
        return tot / iters * 1e3
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3   # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--which", default="bwd,bwd1,bwdacc,fwd,fwd1")
    ap.add_argument("--cold", action="store_true", help="evict the caches before every call")
    a = ap.parse_args()
    global FLUSH
    if a.cold:
        FLUSH = torch.zeros(128 << 20, device="cuda:0")
    dev = torch.device("cuda:0")
    st = nat.stream()
    tag = os.path.basename(os.environ.get("L3U_LIB", "default"))
    for (N, C, L) in SHAPES:
        D = H = W = L
        S = D * H * W
        x = torch.rand(N, C, S, device=dev)
        dz = torch.rand(N, C, S, device=dev)
        dx = torch.zeros(N, C, S, device=dev)
        w = torch.rand(C, 27, device=dev)
        rec = torch.rand(N * C, 8, device=dev)
        nch = nat.query("l3u_dw3_nchunk", N, C, D, H, W)
        dwp = torch.empty(C * N * nch * 27, device=dev)
        inp = torch.empty(C * N * nch * 2, dtype=torch.float64, device=dev)
        u = 4 * N * C * S
        for kind in a.which.split(","):
            if kind.startswith("bwd"):
                r = rec.data_ptr() if kind == "bwd1" else None
                acc = 1 if kind == "bwdacc" else 0
                nb = (4 if acc else 3) * u

                def fn():
                    nat.call("l3u_dw3_bwd", dz.data_ptr(), C * S, x.data_ptr(), C * S, w.data_ptr(),
                             r, dx.data_ptr(), C * S, acc, dwp.data_ptr(),
                             inp.data_ptr() if r else None, N, C, D, H, W, st)
            elif kind == "fwd1s":
                # IN-fused forward with the record finalized in-kernel from GEMM partials, as in
                # the step (nsb partials per (n, c) in the l3u_pw_fwd format)
                nsb = nat.query("l3u_pw_stat_nsb", C, C, S)
                part = torch.empty(N, C, nsb, 3, device=dev)
                part[..., 0] = 64.0
                part[..., 1] = torch.rand(N, C, nsb, device=dev)
                part[..., 2] = 64.0 * torch.rand(N, C, nsb, device=dev)
                gb = torch.rand(2, C, device=dev)
                src = nat.NormSrc(part.data_ptr(), nsb, 1, gb[0].data_ptr(), gb[1].data_ptr(), 0.0,
                                  0x5EED, None, None)
                sp = nat.norm_src_ptr(src)
                nb = 2 * u

                def fn():
                    nat.call("l3u_dw3_fwd", x.data_ptr(), C * S, w.data_ptr(), None, sp,
                             dx.data_ptr(), C * S, N, C, D, H, W, st)
            else:
                r = rec.data_ptr() if kind == "fwd1" else None
                nb = 2 * u

                def fn():
                    nat.call("l3u_dw3_fwd", x.data_ptr(), C * S, w.data_ptr(), r, None,
                             dx.data_ptr(), C * S, N, C, D, H, W, st)
            us = timeit(fn, a.iters)
            print(f"{tag:24s} {kind:7s} [{N},{C},{L}^3] {us:8.2f} us  {nb / us / 1e3:7.0f} GB/s "
                  f"({nb / us / 1e3 / 8000:.3f} of 8 TB/s)", flush=True)


if __name__ == "__main__":
    main()
