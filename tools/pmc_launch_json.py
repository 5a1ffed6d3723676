"""Per-launch counters of one eager training step from tools/pmc_step.sh (FETCH_SIZE, WRITE_SIZE)
and tools/pmc_gemm.sh (SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE) passes.

  traffic   = FETCH_SIZE x 2 (the gfx950 correction, MI355X_MICROARCH.md) + WRITE_SIZE, bytes
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs): rocprofv3's own
              MfmaUtil expression, with GRBM_GUI_ACTIVE's per-XCD sum reduced to the max
Steps end at each adamw launch; the last complete step is reported, in launch order.

    python tools/pmc_launch_json.py <pmc_step dir> <pmc_gemm dir> <out.json>
"""
import csv
import json
import re
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from treehash import product_tree  # noqa: E402


def launches(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = []
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
        out.append({"kernel": name, "grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                    "value": float(r["Counter_Value"]),
                    "dur_us": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3})
    return out


def last_step(seq):
    ends = [i for i, x in enumerate(seq) if "adamw" in x["kernel"]]
    return seq[ends[-2] + 1:ends[-1] + 1]


def main():
    ds, dg, out = sys.argv[1:4]
    f = last_step(launches(f"{ds}/FETCH_SIZE/run_counter_collection.csv", "FETCH_SIZE"))
    w = last_step(launches(f"{ds}/WRITE_SIZE/run_counter_collection.csv", "WRITE_SIZE"))
    mb = last_step(launches(f"{dg}/p1/run_counter_collection.csv", "SQ_VALU_MFMA_BUSY_CYCLES"))
    gui = last_step(launches(f"{dg}/p2/run_counter_collection.csv", "GRBM_GUI_ACTIVE"))
    names = [x["kernel"] for x in f]
    for seq in (w, mb, gui):
        assert [x["kernel"] for x in seq] == names, "passes disagree on the launch sequence"
    items = []
    for a, b, c, g in zip(f, w, mb, gui):
        cyc = g["value"] / 8.0
        items.append({"kernel": a["kernel"], "grid": a["grid"], "wg": a["wg"],
                      "fetch_x2": 2 * a["value"] * 1024, "write": b["value"] * 1024,
                      "traffic": 2 * a["value"] * 1024 + b["value"] * 1024,
                      "mfma_busy_cycles": c["value"], "gui_cycles": cyc,
                      "mfma_util": c["value"] / (cyc * 1024) if cyc > 0 else 0.0,
                      "pmc_dur_us": round(g["dur_us"], 2)})
    tot = sum(i["traffic"] for i in items)
    rec = {"what": "per-launch HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) and MFMA busy fraction "
                   "(SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)) of one eager bs-4 "
                   "48^3 training step, separate rocprofv3 passes", "launches": len(items),
           "step_traffic_bytes": tot, "items": items}
    rec["tree"] = product_tree()
    json.dump(rec, open(out, "w"), indent=1)
    print(f"{len(items)} launches, {tot / 1e9:.3f} GB per step")
    for i, it in enumerate(items):
        print(f"{i:3d} {it['traffic'] / 1e6:8.1f} MB (f {it['fetch_x2'] / 1e6:7.1f} w {it['write'] / 1e6:7.1f}) "
              f"mfma {100 * it['mfma_util']:5.1f}%  {it['kernel'][:58]}")


if __name__ == "__main__":
    main()
