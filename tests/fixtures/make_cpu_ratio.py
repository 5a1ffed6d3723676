"""Equivalence check of the CPU baseline: the oracle restatement
(oracle/unet_oracle.py, the `cpu_baseline` leg of bench.py) against the REFERENCE model, on the
same host cores, the same weights and the same inputs.

Run here (where /root/reference exists) with
    PYTHONDONTWRITEBYTECODE=1 python tests/fixtures/make_cpu_ratio.py
It imports the reference's unet3d.py / losses.py BY FILE PATH, exactly as
tests/golden/make_goldens.py does, and writes tests/fixtures/cpu_ratio.json (data only).

Recorded:
  - parity at dropout 0: max |out_oracle - out_ref|, |loss| difference and the global relative
    gradient error (fp32 both sides, same state_dict);
  - timing: the full train step (fwd + FocalTversky + bwd + AdamW, Dropout3d p=0.1, the bench
    workload bs 4 x 48^3 fp32) of each side, interleaved A/B/A/B on the same threads so drift in
    the host's clock hits both; ratio = oracle ms / reference ms (1.0 = the oracle is a fair
    stand-in for the reference as the CPU baseline).
"""
import importlib.util
import json
import os
import platform
import sys
import time

sys.dont_write_bytecode = True

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import unet_oracle as U  # noqa: E402

REF = os.environ.get("L3U_REFERENCE", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cpu_ratio.json")


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def cpu_model():
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    return platform.processor()


def main():
    unet3d = _load("ref_unet3d", "light_unet/models/unet3d.py")
    losses = _load("ref_losses", "light_unet/models/losses.py")
    threads = int(os.environ.get("THREADS", os.cpu_count() or 1))
    torch.set_num_threads(threads)
    bs, size, drop_p = int(os.environ.get("BS", 4)), int(os.environ.get("SIZE", 48)), 0.1
    warm, steps = 3, int(os.environ.get("STEPS", 10))
    rng = np.random.default_rng(42)
    x = torch.from_numpy(rng.random((bs, 1, size, size, size), dtype=np.float32))
    t = torch.from_numpy((rng.random((bs, 1, size, size, size)) > 0.97).astype(np.float32))
    crit = losses.get_loss_function({"name": "FocalTverskyLoss", "alpha": 0.7, "beta": 0.3,
                                     "gamma": 0.75})

    # ---- parity at dropout 0 (Dropout3d's RNG stream cannot be matched), same weights
    torch.manual_seed(42)
    ref0 = unet3d.Lightweight3DUNet(dropout_p=0.0).train()
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in ref0.state_dict().items()}
    out_r = ref0(x)
    loss_r = crit(out_r, t)
    loss_r.backward()
    out_o = U.unet_forward(sd, x)
    loss_o = U.focal_tversky(out_o, t)
    loss_o.backward()
    num = den = 0.0
    for k, p in ref0.named_parameters():
        d = (sd[k].grad - p.grad).double()
        num += float((d * d).sum())
        den += float((p.grad.double() ** 2).sum())
    parity = {"max_abs_out": float((out_o - out_r).abs().max()),
              "abs_loss": abs(float(loss_o) - float(loss_r)),
              "grad_rel_l2": (num / den) ** 0.5}

    # ---- timing: the bench's train step on each side, interleaved
    torch.manual_seed(42)
    ref = unet3d.Lightweight3DUNet(dropout_p=drop_p).train()
    opt_r = torch.optim.AdamW(ref.parameters(), lr=1e-4, weight_decay=1e-5)
    sdo = {k: v.detach().clone().requires_grad_(True) for k, v in ref.state_dict().items()}
    opt_o = torch.optim.AdamW(list(sdo.values()), lr=1e-4, weight_decay=1e-5)
    blocks = [k[:-len("norm1.weight")] for k in sdo if k.endswith("norm1.weight")]
    g = torch.Generator().manual_seed(0)

    def step_ref():
        loss = crit(ref(x), t)
        opt_r.zero_grad()
        loss.backward()
        opt_r.step()

    def step_oracle():
        masks = {b: (torch.rand(bs, sdo[b + "norm1.weight"].shape[0], generator=g) >= drop_p).float()
                 for b in blocks}
        loss = U.focal_tversky(U.unet_forward(sdo, x, drop_masks=masks, drop_p=drop_p), t)
        opt_o.zero_grad()
        loss.backward()
        opt_o.step()

    for _ in range(warm):
        step_ref()
        step_oracle()
    tr, to = [], []
    for _ in range(steps):
        t0 = time.perf_counter()
        step_ref()
        t1 = time.perf_counter()
        step_oracle()
        t2 = time.perf_counter()
        tr.append(t1 - t0)
        to.append(t2 - t1)
    ms_r, ms_o = 1000 * float(np.median(tr)), 1000 * float(np.median(to))
    rec = {"workload": f"train step bs={bs} {size}^3 fp32, Dropout3d p={drop_p}, AdamW",
           "threads": threads, "cpu_model": cpu_model(), "warmup": warm, "steps": steps,
           "reference_ms_per_step_median": round(ms_r, 2),
           "oracle_ms_per_step_median": round(ms_o, 2),
           "reference_ms_per_step_all": [round(1000 * v, 2) for v in tr],
           "oracle_ms_per_step_all": [round(1000 * v, 2) for v in to],
           "ratio_oracle_over_reference": round(ms_o / ms_r, 4),
           "parity_dropout0": parity, "torch": torch.__version__}
    with open(OUT, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
