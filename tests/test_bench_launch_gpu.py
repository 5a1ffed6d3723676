"""bench.py's own multi-rank launcher: a plain `python bench.py --gpus N` (no WORLD_SIZE in the
environment, the driver's command form) starts the N ranks itself through torch.distributed.run
and relays rank 0's JSON line."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_launcher_command_without_world_size(monkeypatch):
    """CPU: with WORLD_SIZE unset and --gpus 2 the parent only spawns the launcher child (it never
    reaches a torch.cuda call) and exits with the child's return code."""
    sys.path.insert(0, ROOT)
    import bench
    seen = {}

    class R:
        returncode = 7

    def fake_run(cmd, env=None, **kw):
        seen["cmd"], seen["env"] = cmd, env
        return R()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(subprocess, "run", fake_run)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2", "--steps", "3"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 7
    cmd = seen["cmd"]
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=2" in cmd and "--master-addr=127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "2", "--steps", "3"]
    assert cmd[-5].endswith("bench.py")


@pytest.mark.gpu
def test_bench_self_launches_two_ranks(cuda):
    """GPU: `python bench.py --gpus 2 --dist-backend gloo --one-device` (both ranks on this GPU)
    prints one JSON line with n_gpus 2, dp2 and a finite loss."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--dist-backend", "gloo", "--one-device", "--no-cpu-baseline",
           "--no-config5", "--no-sliding", "--no-grouped", "--no-bf16", "--no-dropin", "--no-data", "--no-exchange"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["config"]["parallelism"] == "dp2"
    assert out["config"]["global_batch"] == 8
    assert out["value"] > 0 and out["final_loss"] == out["final_loss"]


def test_paired_call_bytes_are_the_two_calls():
    """CPU: the in-step byte model of a paired GEMM backward launch (l3u_pw_bwd2,
    l3u_pw_bwd_tail_pair) is the sum of the two calls it replaces, so pairing does not move the
    GEMM family's algorithmic bytes."""
    sys.path.insert(0, ROOT)
    import bench
    N, J, S, Ka, Kb = 4, 64, 1728, 64, 32
    p = 1   # any non-null pointer
    one = lambda K, acc: bench.call_bytes(  # noqa: E731
        "l3u_pw_bwd", (p, J * S, None, 0, None, None, 0, p, K * S, p, p, K * S, acc, p, N, J, K, S, p))[2]
    pair = bench.call_bytes("l3u_pw_bwd2", (p, J * S, p, Ka * S, p, p, Ka * S, 0, p, Ka,
                                            p, J * S, p, Kb * S, p, p, Kb * S, 0, p, Kb, N, J, S, p))
    assert pair[0] == "gemm" and pair[2] == one(Ka, 0) + one(Kb, 0)
    J, S, Ka, Kb = 16, 110592, 16, 32
    tail = lambda yr, sel, K, acc: bench.call_bytes(  # noqa: E731
        "l3u_pw_bwd_tail", (p, J * S, p, J * S, yr, J * S, p, p, 4, sel, p, K * S, p, p, K * S, acc, p,
                            N, J, K, S, p))[2]
    args = (p, J * S, None, None, 0, None, 0, 0, p, J * S, p, 4,
            p, J * S, p, p, Ka * S, p, p, Ka * S, 0, p, Ka, 1,
            p, J * S, p, p, Kb * S, p, p, Kb * S, 0, p, Kb, 2, N, J, S, p)
    tp = bench.call_bytes("l3u_pw_bwd_tail_pair", args)
    assert tp[0] == "gemm" and tp[2] == tail(p, 1, Ka, 0) + tail(p, 2, Kb, 0)


def test_reduce_call_bytes(monkeypatch):
    """CPU: the byte model of the weight-gradient reduction launch reads every partial once (fp32,
    fp64 for the InstanceNorm affine partials) and the item table, and per output writes the
    gradient and (the fused AdamW form) reads and writes the parameter and both moments."""
    sys.path.insert(0, ROOT)
    import bench
    items = [[0, 1728, 512, 1, 32, 0, 0, 0], [64, 4, 3, 12, 16, 32, 0, 1]]
    monkeypatch.setattr(bench, "SEG_ITEMS", {99: items})
    f, label, b = bench.call_bytes("l3u_reduce_segments_adamw", (1, 99, 2))
    assert f == "reduce" and "2 items" in label
    assert b == 1728 * 32 * 4 + 4 * 16 * 8 + 2 * 64 + 28 * 48
    assert bench.call_bytes("l3u_reduce_segments", (1, 99, 2))[2] == 1728 * 32 * 4 + 4 * 16 * 8 + 2 * 64 + 4 * 48
    assert bench.call_bytes("l3u_reduce_segments", (1, 98, 2)) is None   # items not recorded
