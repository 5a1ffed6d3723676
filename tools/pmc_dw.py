"""Driver for the rocprofv3 PMC passes of the dominant call (tools/pmc.sh): l3u_dw3_bwd at the
bench shape [4, 32, 48^3] (up3.res_block.conv1.depthwise), 10 calls."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402

N, C, L = 4, 32, 48
S = L ** 3
dev = torch.device("cuda:0")
x = torch.rand(N, C, S, device=dev)
dz = torch.rand(N, C, S, device=dev)
dx = torch.zeros_like(x)
ACC = 1   # the step's call adds to the shortcut's d(input) (l3u_pw_bwd_tail_pair runs first)
w = torch.rand(C, 27, device=dev)
nch = nat.query("l3u_dw3_nchunk", N, C, L, L, L)
dwp = torch.empty(C * N * nch * 27, device=dev)
for _ in range(10):
    nat.call("l3u_dw3_bwd", dz.data_ptr(), C * S, x.data_ptr(), C * S, w.data_ptr(), None,
             dx.data_ptr(), C * S, ACC, dwp.data_ptr(), None, N, C, L, L, L, nat.stream())
torch.cuda.synchronize()
print("done", flush=True)
