"""Stage timestamps of l3u_sblock_fwd (a library built with -DL3U_SB_PROF, tools/mkvar.sh):
per-stage mean / max over workgroups, in microseconds (wall_clock64 runs at 100 MHz)."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "light-3d-unet-front_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from light_unet import _native as nat  # noqa: E402

NAMES = ["x stage", "dw1+W", "barrier1", "z1 stage", "pw1", "stats1", "dw2+W", "barrier2",
         "z2 stage", "pw2", "stats2", "out"]


def run(N, Cin, Cout, D, H, W, sc):
    dev = torch.device("cuda:0")
    S = D * H * W
    g = torch.Generator().manual_seed(1)
    r = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    P = dict(x=r(N, Cin, S), wdw1=r(Cin, 27), wpw1=r(Cout, Cin), wdw2=r(Cout, 27), wpw2=r(Cout, Cout),
             g1=r(Cout), b1=r(Cout), g2=r(Cout), b2=r(Cout))
    if sc:
        P.update(wsc=r(Cout, Cin), gsc=r(Cout), bsc=r(Cout))
    o = {k: torch.empty(N, c, S, device=dev) for k, c in
         (("z1", Cin), ("y1", Cout), ("z2", Cout), ("y2", Cout), ("r", Cout), ("out", Cout))}
    recs = torch.empty(3, N, Cout, 8, device=dev)
    G = Cout // 16
    sync = torch.zeros(64 + N * G * 32, dtype=torch.int32, device=dev)
    p = lambda k: P[k].data_ptr() if k in P else None  # noqa: E731
    a = nat.SblockFwdArgs(P["x"].data_ptr(), Cin * S, p("wdw1"), p("wpw1"), p("wsc"), p("gsc"), p("bsc"),
                          p("g1"), p("b1"), p("wdw2"), p("wpw2"), p("g2"), p("b2"), 0.1, 1, 5, None,
                          o["z1"].data_ptr(), o["y1"].data_ptr(), o["z2"].data_ptr(), o["y2"].data_ptr(),
                          o["r"].data_ptr() if sc else None, o["out"].data_ptr(), Cout * S,
                          recs[0].data_ptr(), recs[1].data_ptr(), recs[2].data_ptr(), sync.data_ptr())
    st = torch.cuda.current_stream().cuda_stream
    res = []
    for it in range(30):
        # a large unrelated write between launches, as in the step (dirty L2 lines)
        junk = torch.ones(8 << 20, device=dev) * it
        nat.call("l3u_sblock_fwd", ctypes.pointer(a), N, Cin, Cout, D, H, W, st)
        torch.cuda.synchronize()
        if it >= 10:
            t = sync[64:].cpu().numpy().view(np.uint64).reshape(N * G, 16)[:, :13].astype(np.int64)
            res.append(t)
        del junk
    t = np.stack(res)                          # [it][blocks][13]
    d = np.diff(t, axis=2) / 100.0             # us
    start_skew = (t[:, :, 0] - t[:, :, 0].min(1, keepdims=True)) / 100.0
    total = (t[:, :, 12].max(1) - t[:, :, 0].min(1)) / 100.0
    print(f"shape N={N} {Cin}->{Cout} {D}x{H}x{W} sc={sc}: in-kernel span {total.mean():.1f} us, "
          f"start skew max {start_skew.max(1).mean():.1f} us, err flag {sync[N].item()}")
    for i, nm in enumerate(NAMES):
        print(f"  {nm:10s} mean {d[:, :, i].mean():6.2f}  max {d[:, :, i].max(1).mean():6.2f}")


if __name__ == "__main__":
    run(4, 64, 128, 6, 6, 6, 1)
    run(4, 128, 128, 6, 6, 6, 0)
