"""Counter driver: the ConvTranspose3d backward (l3u_convt_bwd_fused) at one model shape, issued
back-to-back `iters` times (rocprofv3 --pmc passes: tools/pmc_kernel.sh).

    python tools/convt_probe.py [N,Ci,Co,L] [iters]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))

import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402


def main():
    N, Ci, Co, L = (int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "4,32,16,24").split(","))
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    Si = L ** 3
    dcat = torch.randn(N, 2 * Co, 8 * Si, device=dev)
    x = torch.randn(N, Ci, Si, device=dev)
    w = torch.randn(Ci, Co * 8, device=dev)
    dx = torch.empty(N, Ci, Si, device=dev)
    P = nat.query("l3u_convt_bwd_fused_nparts", N, Ci, Co, L, L, L)
    wp, bp = torch.empty(P * Ci * Co * 8, device=dev), torch.empty(P * Co, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(iters):
        nat.call("l3u_convt_bwd_fused", dcat.data_ptr(), 2 * Co * 8 * Si, x.data_ptr(), Ci * Si, w.data_ptr(),
                 dx.data_ptr(), Ci * Si, wp.data_ptr(), bp.data_ptr(), N, Ci, Co, L, L, L, st)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
