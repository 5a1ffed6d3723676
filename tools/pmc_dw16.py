"""Driver for the SQ counter passes (tools/pmc_sq.sh with PMC_DRIVER=tools/pmc_dw16.py) of the
[4,16,48^3] depthwise launches of the step: l3u_dw3_bwd (plain and IN-fused, rec + in_part) and the
IN-fused l3u_dw3_fwd, 10 calls each."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

N, C, L = 4, 16, 48
S = L ** 3
dev = torch.device("cuda:0")
x = torch.rand(N, C, S, device=dev)
dz = torch.rand(N, C, S, device=dev)
dx = torch.empty_like(x)
w = torch.rand(C, 27, device=dev)
rec = torch.zeros(N * C, 8, device=dev)
rec[:, 1] = 1.0
rec[:, 2] = 1.0
rec[:, 4] = 1.0
rec[:, 5] = 1.0
nch = nat.query("l3u_dw3_nchunk", N, C, L, L, L)
dwp = torch.empty(C * N * nch * 27, device=dev)
inp = torch.empty(C * N * nch * 2, dtype=torch.float64, device=dev)
for _ in range(10):
    nat.call("l3u_dw3_bwd", dz.data_ptr(), C * S, x.data_ptr(), C * S, w.data_ptr(), None,
             dx.data_ptr(), C * S, 0, dwp.data_ptr(), None, N, C, L, L, L, nat.stream())
for _ in range(10):
    nat.call("l3u_dw3_bwd", dz.data_ptr(), C * S, x.data_ptr(), C * S, w.data_ptr(), rec.data_ptr(),
             dx.data_ptr(), C * S, 0, dwp.data_ptr(), inp.data_ptr(), N, C, L, L, L, nat.stream())
for _ in range(10):
    nat.call("l3u_dw3_fwd", x.data_ptr(), C * S, w.data_ptr(), rec.data_ptr(), None, dx.data_ptr(), C * S,
             N, C, L, L, L, nat.stream())
torch.cuda.synchronize()
print("done", flush=True)
