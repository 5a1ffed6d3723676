"""Accuracy of the in-kernel InstanceNorm record merge (l3u_in_finalize) vs an fp64 host merge."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402
from light_unet import _native as nat  # noqa: E402
dev = torch.device("cuda:0")
for nsb, cnt, mu0 in ((128, 256, 0.3), (432, 256, 5.0), (27, 64, 0.01), (1, 4096, 1.0)):
    N, C = 4, 64
    vals = torch.randn(N, C, nsb, cnt, dtype=torch.float64) * 0.7 + mu0
    vals = vals.float().double()
    part = torch.stack([torch.full((N, C, nsb), float(cnt), dtype=torch.float64), vals.mean(-1),
                        ((vals - vals.mean(-1, keepdim=True)) ** 2).sum(-1)], -1).float()
    pd = part.to(dev).contiguous()
    rec = torch.empty(N * C * 8, device=dev)
    nat.call("l3u_in_finalize", pd.data_ptr(), nsb, None, None, 0.0, 1, None, 0, rec.data_ptr(), N, C,
             nat.stream())
    torch.cuda.synchronize()
    r = rec.view(N, C, 8).double().cpu()
    flat = vals.reshape(N, C, -1)
    mean, var = flat.mean(-1), flat.var(-1, unbiased=False)
    rstd = 1 / torch.sqrt(var + 1e-5)
    em = ((r[..., 0] - mean).abs() / mean.abs().clamp_min(1e-3)).max().item()
    er = ((r[..., 1] - rstd).abs() / rstd).max().item()
    print(f"nsb {nsb:4d} cnt {cnt:5d} mean {mu0}: mean rel err {em:.3e}  rstd rel err {er:.3e}")
