"""Dump the bf16 engine's stored forward activations (per block z1, y1, r, z2, y2, out and the
records) and the output / parameter gradients of one FocalTversky step on a golden fixture, for
a per-tensor comparison with oracle/bf16_oracle.py on the CPU.

    python tools/bf16_dump.py model_b2_32.npz gpurun_out/bf16_dump.npz
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "light-3d-unet-front_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from light_unet.models.losses import FocalTverskyLoss  # noqa: E402
from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402


def main():
    z = np.load(os.path.join(ROOT, "tests", "golden", sys.argv[1]))
    dev = torch.device("cuda:0")
    m = Lightweight3DUNet(dropout_p=0.0, compute_dtype=torch.bfloat16)
    m.load_state_dict({k[2:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("w/")})
    m = m.to(dev).train()
    x = torch.from_numpy(z["x"]).to(dev)
    t = torch.from_numpy(z["target"]).to(dev)
    eng = m.engine
    eng.set_act_dtype(torch.bfloat16)
    p, sv = eng.forward(m.flat_parameters(), x, training=True, dropout_p=0.0, save=True)
    torch.cuda.synchronize()
    out = {"p": p.float().cpu().numpy()}

    for pre, b in sv["blk"].items():
        for key in ("z1", "y1", "z2", "y2"):
            if key in b and b[key] is not None:
                out[f"{pre}{key}"] = b[key].float().cpu().numpy()
        d, h, w = b["dims"]
        S = d * h * w
        for key in ("r", "out", "x"):
            v = b.get(key)
            if v is None:
                continue
            flat = v.t.reshape(-1)
            N = x.shape[0]
            out[f"{pre}{key}"] = torch.stack(
                [flat[n * v.ns + v.off: n * v.ns + v.off + v.C * S] for n in range(N)]).float().cpu().numpy()
        out[f"{pre}recs"] = b["recs"].cpu().numpy()
    loss = FocalTverskyLoss()(m(x), t)
    m.zero_grad(set_to_none=True)
    loss.backward()
    torch.cuda.synchronize()
    out["loss"] = np.array(loss.item())
    for k, prm in m.named_parameters():
        out["g/" + k] = prm.grad.cpu().numpy()
    np.savez_compressed(sys.argv[2], **out)
    print("saved", len(out), "arrays")


if __name__ == "__main__":
    main()
