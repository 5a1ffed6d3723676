"""The data-parallel training step on a real RCCL process group (backend "nccl", one rank on the
one-GPU box): RCCL initialisation, the fp64 FocalTversky sums all-reduce, the flat-gradient
all-reduce, the three graph segments with eager collectives and the collectives captured inside
the graph -- each checked against the one-process single-graph step (fused gradient
reduction + AdamW) on the same weights and batches.  The probe (tools/rccl_probe.py) runs in
its own process so that this test session never holds a process group."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_rccl_one_rank_step_matches_single_graph(cuda, tmp_path):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RCCL_SIZE="48")
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "rccl_probe.py"), str(tmp_path),
                        str(port)], capture_output=True, text=True, timeout=110, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.load(open(tmp_path / "rccl.json"))
    print(rec)
    assert rec["backend"] == "nccl" and rec["world"] == 1
    z = np.load(tmp_path / "rccl.npz")
    for form in ("segmented", "captured"):
        for i in range(3):
            ls, lf = float(z[f"single_loss{i}"]), float(z[f"{form}_loss{i}"])
            # the sums reach the loss through l3u_ftl_reduce + the all-reduce instead of the
            # out_conv backward's own reduction: the same fp64 sums, so the same fp32 loss
            assert abs(lf - ls) <= 1e-6 * abs(ls), (form, i, lf, ls)
            ps, pf = z[f"single_p{i}"].astype(np.float64), z[f"{form}_p{i}"].astype(np.float64)
            # a one-rank all-reduce returns its input, and the separate update launch applies the
            # fused launch's per-element arithmetic: the trajectories agree to fp32 rounding
            assert np.abs(pf - ps).max() <= 1e-6, (form, i, np.abs(pf - ps).max())
    # the captured collectives replay in the same graph as the step: nothing is left eager
    assert rec["ms_per_step"]["captured"] > 0
