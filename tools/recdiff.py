"""Per-sample determinism across batch sizes: the forward of samples 0..1 inside a bs-4 batch vs
a bs-2 batch must give bitwise-equal InstanceNorm records and outputs (every op is per sample)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(42)
L = int(os.environ.get("RD_SIZE", "32"))
m = Lightweight3DUNet(dropout_p=0.0).to(dev)
eng, flat = m.engine, m._flat
x = torch.rand(4, 1, L, L, L, device=dev)
outs = []
for bs in (4, 2):
    p, sv = eng.forward(flat, x[:bs].contiguous(), training=True, save=True)
    torch.cuda.synchronize()
    outs.append((p.clone(), {k: v["recs"].clone().view(3, bs, -1, 8) for k, v in sv["blk"].items()}))
(p4, r4), (p2, r2) = outs
print("prob max diff", (p4[:2] - p2).abs().max().item())
for k in r4:
    d = (r4[k][:, :2] - r2[k]).abs()
    print(f"{k:22s} rec max diff {d.max().item():.3e}  (mean {d[..., 0].max().item():.2e} rstd {d[..., 1].max().item():.2e})")
