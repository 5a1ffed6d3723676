"""Per-launch SQ counters of one eager training step from tools/pmc_sq_step.sh's passes (the last
complete step: steps end at each AdamW launch), with the derived figures used in DESIGN §8:

  waves_per_simd  mean resident waves per SIMD over the launch: SQ_WAVE_CYCLES counts quad-cycles
                  summed over every wave, SQ_BUSY_CYCLES counts cycles summed over the 32 shader
                  engines (busy / 32 = the launch's duration in cycles: 28-33 x the rocprof
                  duration in us at the ~2.1-2.4 GHz clock, r4g records), so
                  waves/SIMD = 4 * WAVE_CYCLES / (BUSY_CYCLES / 32) / 1024 SIMDs
                  = WAVE_CYCLES / BUSY_CYCLES / 8  (round 4's field omitted the 4 * 32 and read
                  ~128x low)
  valu_busy       SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (per wave: the share of its life issuing VALU)
  wait_frac       SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked on s_waitcnt / barrier)
  salu_per_valu   SQ_INSTS_SALU / SQ_INSTS_VALU
  valu_per_wave   SQ_INSTS_VALU / SQ_WAVES

    python tools/sq_step_json.py <pmc_sq_step out dir> <out.json>
"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from treehash import product_tree  # noqa: E402


def launches(path):
    """[(kernel, grid, dur_us, {counter: value})] in dispatch order."""
    by = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
        e = by.setdefault(d, [name, int(r.get("Grid_Size", 0) or 0), 0.0, {}])
        e[3][r["Counter_Name"]] = float(r["Counter_Value"])
        if "End_Timestamp" in r and r["End_Timestamp"]:
            e[2] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return [tuple(by[k]) for k in sorted(by)]


def last_step(seq):
    ends = [i for i, x in enumerate(seq) if "adamw" in x[0]]
    return seq[ends[-2] + 1:ends[-1] + 1]


def main():
    d, out = sys.argv[1], sys.argv[2]
    passes = []
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        f = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
        if f:
            passes.append(last_step(launches(f[0])))
    names = [x[0] for x in passes[0]]
    for q in passes[1:]:
        assert [x[0] for x in q] == names, "passes disagree on the launch sequence"
    items = []
    for i, name in enumerate(names):
        c = {}
        for q in passes:
            c.update(q[i][3])
        wc = c.get("SQ_WAVE_CYCLES", 0.0)
        it = {"kernel": name, "grid": passes[0][i][1],
              "pmc_dur_us": round(sum(q[i][2] for q in passes) / len(passes), 2), "counters": c}
        if wc > 0 and c.get("SQ_BUSY_CYCLES", 0) > 0:
            it["waves_per_simd"] = round(4.0 * wc / (c["SQ_BUSY_CYCLES"] / 32.0) / 1024, 2)
            it["valu_busy"] = round(c.get("SQ_ACTIVE_INST_VALU", 0) / wc, 3)
            it["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0) / wc, 3)
        if c.get("SQ_INSTS_VALU", 0) > 0:
            it["salu_per_valu"] = round(c.get("SQ_INSTS_SALU", 0) / c["SQ_INSTS_VALU"], 3)
            it["valu_per_wave"] = round(c["SQ_INSTS_VALU"] / max(c.get("SQ_WAVES", 1), 1), 1)
        items.append(it)
    rec = {"what": "SQ counters per launch of one eager bs-4 training step (rocprofv3 --pmc, two "
                   "passes, kernel-trace only)", "tree": product_tree(), "launches": len(items),
           "items": items}
    json.dump(rec, open(out, "w"), indent=1)
    for it in items:
        print(f"{it['pmc_dur_us']:7.1f} us  w/simd {it.get('waves_per_simd', 0):5.2f}  valu {it.get('valu_busy', 0):5.3f}  "
              f"wait {it.get('wait_frac', 0):5.3f}  salu/valu {it.get('salu_per_valu', 0):5.3f}  "
              f"valu/wave {it.get('valu_per_wave', 0):7.1f}  {it['kernel'][:58]}")


if __name__ == "__main__":
    main()
