"""Fused l3u_dwpw_fwd vs the unfused l3u_dw3_fwd -> l3u_pw_fwd(2) launches at the model's shapes
(us per call, algorithmic GB/s).  python tools/dwpw_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from kbench import timeit  # noqa: E402

dev = torch.device("cuda:0")
st = nat.stream()
# (N, K, J, L, shortcut, xf)
for N, K, J, L, sc, xf in [(4, 16, 16, 48, 0, 1), (4, 16, 16, 48, 0, 2), (4, 16, 16, 48, 0, 0),
                          (4, 16, 32, 24, 1, 0)]:
    D = H = W = L
    S = D * H * W
    x = torch.rand(N, K, S, device=dev)
    wdw, wpw, wsc = torch.rand(K, 27, device=dev), torch.rand(J, K, device=dev), torch.rand(J, K, device=dev)
    y, r, z = torch.empty(N, J, S, device=dev), torch.empty(N, J, S, device=dev), torch.empty(N, K, S, device=dev)
    nsbp = nat.query("l3u_pw_stat_nsb", K, K, S)
    part = torch.empty(N, K, nsbp, 3, device=dev)
    part[..., 0] = 64.0
    part[..., 1] = torch.rand(N, K, nsbp, device=dev)
    part[..., 2] = 64.0 * torch.rand(N, K, nsbp, device=dev)
    gb = torch.rand(2, K, device=dev)
    src = nat.NormSrc(part.data_ptr(), nsbp, 1, gb[0].data_ptr(), gb[1].data_ptr(), 0.0, 0x5EED, None, None)
    sp = nat.norm_src_ptr(src) if xf == 1 else None
    recp = torch.rand(N * K * 8, device=dev).data_ptr() if xf == 2 else None
    nsb = nat.query("l3u_dwpw_stat_nsb", K, J, D, H, W)
    ys, rs = torch.empty(N * J * nsb * 3, device=dev), torch.empty(N * J * nsb * 3, device=dev)
    nsb2 = nat.query("l3u_pw_stat_nsb", K, J, S)
    ys2, rs2 = torch.empty(N * J * nsb2 * 3, device=dev), torch.empty(N * J * nsb2 * 3, device=dev)

    def fused():
        nat.call("l3u_dwpw_fwd", x.data_ptr(), K * S, wdw.data_ptr(), recp, sp, wpw.data_ptr(),
                 y.data_ptr(), J * S, ys.data_ptr(), wsc.data_ptr() if sc else None,
                 r.data_ptr() if sc else None, J * S, rs.data_ptr() if sc else None, z.data_ptr(),
                 K * S, N, K, J, D, H, W, st)

    def unfused():
        nat.call("l3u_dw3_fwd", x.data_ptr(), K * S, wdw.data_ptr(), recp, sp, z.data_ptr(), K * S,
                 N, K, D, H, W, st)
        if sc:
            nat.call("l3u_pw_fwd2", x.data_ptr(), K * S, wsc.data_ptr(), r.data_ptr(), J * S,
                     rs2.data_ptr(), z.data_ptr(), K * S, wpw.data_ptr(), y.data_ptr(), J * S,
                     ys2.data_ptr(), N, K, J, S, st)
        else:
            nat.call("l3u_pw_fwd", z.data_ptr(), K * S, wpw.data_ptr(), 0, None, y.data_ptr(), J * S,
                     0, ys2.data_ptr(), N, K, J, S, st)
    ub = 4 * N * S
    fb = ub * (K + K + J * (1 + sc))            # x read, z written, y (+ r) written
    nb = ub * (K + K + K + K * (sc) + J * (1 + sc))   # + z re-read (+ x re-read by the shortcut)
    tf, tu = timeit(fused, 50), timeit(unfused, 50)
    print(f"{os.path.basename(os.environ.get('L3U_LIB', 'default'))} [{N},{K}->{J},{L}^3] sc={sc} xf={xf}: fused {tf:7.2f} us ({fb / tf / 1e3:6.0f} GB/s, "
          f"{fb / tf / 8e6:.3f}) | unfused {tu:7.2f} us ({nb / tu / 1e3:6.0f} GB/s)", flush=True)
