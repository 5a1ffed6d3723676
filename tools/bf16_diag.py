"""bf16 network vs fp32 HIP path vs the reference's fp64 goldens: output error statistics and
thresholded-mask agreement (diagnostic for tests/test_bf16_gpu.py bounds)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    for fname in ("model_b2_32.npz", "model_b1_48.npz", "model_c32_b1_64.npz"):
        z = np.load(os.path.join(ROOT, "tests", "golden", fname))
        enc = [32, 64, 128, 256] if "c32" in fname else [16, 32, 64, 128]
        outs = {}
        for dt in (torch.float32, torch.bfloat16):
            m = Lightweight3DUNet(encoder_channels=enc, dropout_p=0.0, compute_dtype=dt)
            m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")})
            m = m.to(dev).eval()
            with torch.no_grad():
                outs[dt] = m(torch.from_numpy(z["x"]).to(dev)).cpu().double().numpy()
        o16, o32 = outs[torch.bfloat16], outs[torch.float32]
        ref = z["out"] if "out" in z.files else o32
        d = np.abs(o16 - ref)
        print(f"{fname}: p range [{ref.min():.4f}, {ref.max():.4f}] std {ref.std():.4f}; |bf16-ref| "
              f"max {d.max():.3e} mean {d.mean():.3e} p99 {np.quantile(d, 0.99):.3e}; |fp32-ref| max "
              f"{np.abs(o32 - ref).max():.2e}")
        for thr in (0.1, 0.3, 0.5, 0.7):
            agree = np.mean((o16 >= thr) == (ref >= thr))
            near = [np.mean(np.abs(ref - thr) < e) for e in (1e-3, 3e-3, 1e-2)]
            print(f"   thr {thr}: agree {agree:.5f}; frac within 1e-3/3e-3/1e-2 of thr: "
                  f"{near[0]:.4f} {near[1]:.4f} {near[2]:.4f}")


if __name__ == "__main__":
    main()
