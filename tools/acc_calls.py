"""Which C-ABI calls of the headline step accumulate into their output (accumulate / acc_* != 0):
prints every pointwise / ConvTranspose3d / depthwise-backward call of one eager step with its
accumulate flags.   python tools/acc_calls.py"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "light-3d-unet-front_amd"))
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402
from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402
from light_unet.train_step import TrainStep  # noqa: E402

hdr = open(os.path.join(ROOT, "include", "l3u.h")).read()
pos = {}
for m in re.finditer(r"int (l3u_\w+)\(([^;]*?)\);", hdr, re.S):
    names = [a.strip().split()[-1].lstrip("*") for a in m.group(2).split(",")]
    idx = [i for i, a in enumerate(names) if a == "accumulate" or a.startswith("acc_")]
    if idx:
        pos[m.group(1)] = [(i, names[i]) for i in idx]
calls = []
orig = nat.call


def spy(name, *a):
    base = name[:-5] if name.endswith("_bf16") else name
    if base in pos:
        calls.append((name, [(n, a[i]) for i, n in pos[base]], a[-6:-1]))
    return orig(name, *a)


dev = torch.device("cuda:0")
torch.manual_seed(0)
m = Lightweight3DUNet(encoder_channels=[16, 32, 64, 128], dropout_p=0.1).to(dev).train()
ts = TrainStep(m, {"alpha": 0.7, "beta": 0.3, "gamma": 0.75}, lr=1e-4, weight_decay=1e-5)
x = torch.rand(4, 1, 48, 48, 48, device=dev)
t = (torch.rand(4, 1, 48, 48, 48, device=dev) > 0.97).float()
ts(x, t)
torch.cuda.synchronize()
nat.call = spy
ts(x, t)
torch.cuda.synchronize()
nat.call = orig
for name, flags, tail in calls:
    print(name, " ".join(f"{n}={v}" for n, v in flags), "shape-tail", tail)
