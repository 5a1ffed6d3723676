"""Dump the weight-gradient reduction items of the bench step (count / length / stride classes)
as JSON, for modelling the l3u_reduce_segments(_adamw) launch.
usage: python tools/items_dump.py OUT.json [--size 48 --batch 4]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "light-3d-unet-front_amd"))
import torch  # noqa: E402


def main():
    out = sys.argv[1]
    size = int(sys.argv[sys.argv.index("--size") + 1]) if "--size" in sys.argv else 48
    batch = int(sys.argv[sys.argv.index("--batch") + 1]) if "--batch" in sys.argv else 4
    from light_unet.models.unet3d import Lightweight3DUNet
    from light_unet.train_step import TrainStep
    dev = torch.device("cuda", 0)
    torch.manual_seed(42)
    model = Lightweight3DUNet(encoder_channels=[16, 32, 64, 128]).to(dev).train()
    step = TrainStep(model, {"alpha": 0.7, "beta": 0.3, "gamma": 0.75}, lr=1e-4, weight_decay=1e-5)
    x = torch.randn(batch, 1, size, size, size, device=dev)
    t = (torch.rand(batch, 1, size, size, size, device=dev) > 0.5).float()
    for _ in range(2):
        step(x, t)
    torch.cuda.synchronize()
    res = {}
    for key, items in model.engine._items.items():
        rows = items.cpu().tolist()
        res[str(key)] = rows
        print(key, len(rows), "items,", sum(r[1] * r[4] * (8 if r[7] else 4) for r in rows) / 1e6,
              "MB of partials")
    with open(out, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
