"""Wave stamps of the graph-replayed training step (profiling variant build, -DL3U_STAMP):
for every launch of at most 65536 waves, when each wave began and ended (wall clock, 10 ns),
so that a launch's time splits into dispatch spread, wave bodies and the boundary to the next.

    bash tools/mkvar.sh stamp -DL3U_STAMP
    L3U_LIB=$PWD/light-3d-unet-front_amd/lib/var_stamp.so python tools/stamp.py [out.json [dump.json]]
    (STAMP_DUMP_ID=<kernel id>: every wave of that kernel in the last replay, with the engine's
    reduction items, into dump.json)

Per launch (in step order): kernel, waves, gap = its first wave begin - the previous stamped
launch's last wave end (the kernel boundary when both are stamped; larger when an unstamped big
launch ran between), spread = last - first wave begin, body = median / max wave duration,
span = last end - first begin.  Median over REPS replays.
"""
import ctypes
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "light-3d-unet-front_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from light_unet import _native as nat  # noqa: E402
from light_unet.models.unet3d import Lightweight3DUNet  # noqa: E402
from light_unet.train_step import TrainStep  # noqa: E402

REPS = 5
CAP = 1 << 20
TICK_US = 0.01   # wall_clock64: 100 MHz


def kernel_names():
    names = {}
    for f in ("pwconv", "dwconv", "norm", "misc", "dwpw", "convt"):
        src = open(os.path.join(ROOT, "light-3d-unet-front_amd", "csrc", f + ".hip")).read()
        for m in re.finditer(r"L3U_STAMP_SCOPE\((\d+)\)", src):
            head = src[:m.start()]
            names[int(m.group(1))] = re.findall(r"void\s+(\w+)\s*\(", head)[-1]
    return names


def launches(rec):
    """Group wave records into launches: stream order means launch k+1's waves all begin after
    launch k's last wave ended."""
    rec = rec[np.argsort(rec["t0"], kind="stable")]
    out, cur = [], None
    for r in rec:
        key = (int(r["id"]), int(r["nwg"]))
        if cur is None or key != cur["key"] or r["t0"] >= cur["t1max"]:
            cur = {"key": key, "t0": [], "t1": [], "m0": [], "m1": [], "t1max": 0}
            out.append(cur)
        if r["m0"]:   # intermediate marks (L3U_STAMP_MARK): stage durations from the wave begin
            cur["m0"].append(int(r["m0"]) - int(r["t0"]))
        if r["m1"]:
            cur["m1"].append(int(r["m1"]) - int(r["t0"]))
        cur["t0"].append(int(r["t0"]))
        cur["t1"].append(int(r["t1"]))
        cur["t1max"] = max(cur["t1max"], int(r["t1"]))
    return out


def main():
    dev = torch.device("cuda:0")
    lib = nat.load()
    lib.l3u_stamp_setup.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
    torch.manual_seed(42)
    m = Lightweight3DUNet(dropout_p=0.1).to(dev).train()
    ts = TrainStep(m, {"alpha": 0.7, "beta": 0.3, "gamma": 0.75}, lr=1e-4, weight_decay=1e-5,
                   distributed=False)
    rng = np.random.default_rng(1)
    x = torch.from_numpy(rng.random((4, 1, 48, 48, 48), dtype=np.float32)).to(dev)
    t = torch.from_numpy((rng.random((4, 1, 48, 48, 48)) > 0.97).astype(np.float32)).to(dev)
    ts.capture(x, t, warmup=2)
    for _ in range(10):
        ts.replay()
    torch.cuda.synchronize()
    dt = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("m0", "<u8"), ("m1", "<u8"), ("id", "<u4"),
                   ("blk", "<u4"), ("nwg", "<u4"), ("pad", "<u4"), ("r0", "<u4"), ("r1", "<u4")])
    buf = torch.zeros(CAP * dt.itemsize, dtype=torch.uint8, device=dev)
    ctr = torch.zeros(256, dtype=torch.int32, device=dev)
    names = kernel_names()
    runs = []
    for _ in range(REPS):
        ctr.zero_()
        buf.zero_()
        torch.cuda.synchronize()
        assert lib.l3u_stamp_setup(buf.data_ptr(), ctr.data_ptr(), CAP) == 0
        ts.replay()
        torch.cuda.synchronize()
        assert lib.l3u_stamp_setup(None, None, 0) == 0
        assert int(ctr.max().item()) <= CAP // 256, int(ctr.max().item())
        rec = np.frombuffer(buf.cpu().numpy().tobytes(), dtype=dt)
        rec = rec[rec["pad"] == 1]   # written slots
        runs.append(launches(rec))
    dump_id = int(os.environ.get("STAMP_DUMP_ID", "0"))
    if dump_id and len(sys.argv) > 2:   # every wave of that kernel in the last replay + the items
        r = rec[rec["id"] == dump_id]
        items = {str(k): v.cpu().tolist() for k, v in m.engine._items.items()}
        with open(sys.argv[2], "w") as f:
            json.dump({"id": dump_id, "blk": r["blk"].tolist(), "t0": r["t0"].tolist(),
                       "t1": r["t1"].tolist(), "items": items}, f)
    nl = min(len(r) for r in runs)
    rows = []
    for i in range(nl):
        g = [r[i] for r in runs]
        row = {"kernel": names.get(g[0]["key"][0], str(g[0]["key"][0])), "workgroups": g[0]["key"][1],
               "waves": len(g[0]["t0"])}
        for k, f in (("spread_us", lambda L: max(L["t0"]) - min(L["t0"])),
                     ("body_med_us", lambda L: float(np.median(np.array(L["t1"]) - np.array(L["t0"])))),
                     ("body_max_us", lambda L: max(np.array(L["t1"]) - np.array(L["t0"]))),
                     ("span_us", lambda L: L["t1max"] - min(L["t0"]))):
            row[k] = round(float(np.median([f(L) for L in g])) * TICK_US, 2)
        for k in ("m0", "m1"):
            if g[0][k]:
                row[k + "_med_us"] = round(float(np.median([np.median(L[k]) for L in g if L[k]])) * TICK_US, 2)
        if i > 0:
            row["gap_us"] = round(float(np.median([min(r[i]["t0"]) - r[i - 1]["t1max"] for r in runs]))
                                  * TICK_US, 2)
        rows.append(row)
    print(f"{'gap':>6} {'spread':>6} {'body50':>6} {'bodymx':>6} {'span':>6}  waves  kernel")
    for r in rows:
        print(f"{r.get('gap_us', 0):6.2f} {r['spread_us']:6.2f} {r['body_med_us']:6.2f} "
              f"{r['body_max_us']:6.2f} {r['span_us']:6.2f} {r['waves']:6d}  {r['kernel']}"
              + (f"  marks {r.get('m0_med_us', '-')} / {r.get('m1_med_us', '-')}" if "m0_med_us" in r or "m1_med_us" in r else ""))
    tot = {k: round(sum(r.get(k, 0) for r in rows), 1) for k in ("gap_us", "span_us")}
    print("stamped launches", len(rows), "sum span", tot["span_us"], "sum gap", tot["gap_us"])
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump({"launches": rows, "totals": tot, "reps": REPS}, f, indent=1)


if __name__ == "__main__":
    main()
