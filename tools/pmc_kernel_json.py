"""Per-kernel mean counters of tools/pmc_kernel.sh's passes (dispatches 3.. of each kernel name,
the first ones warm the caches), with the derived figures:
  mfma_util  SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)
  traffic    FETCH_SIZE x 2 (gfx950 correction) + WRITE_SIZE, bytes
    python tools/pmc_kernel_json.py <dir> <out.json>"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from treehash import product_tree  # noqa: E402


def main():
    d, out = sys.argv[1], sys.argv[2]
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "p*", "**", "*counter_collection.csv"), recursive=True)):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        seen = collections.Counter()
        for r in rows:
            k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
            if r["Counter_Name"] == rows[0]["Counter_Name"] or True:
                seen[(k, r["Dispatch_Id"])] += 0
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r.get("End_Timestamp"):
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    res = {}
    for k, cs in acc.items():
        m = {c: sum(v[2:]) / max(len(v[2:]), 1) for c, v in cs.items()}
        it = {"counters": m}
        if dur[k]:
            it["pmc_dur_us"] = round(sum(dur[k][2:]) / max(len(dur[k][2:]), 1), 2)
        if m.get("GRBM_GUI_ACTIVE"):
            it["mfma_util"] = round(m.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (m["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
        if "FETCH_SIZE" in m:
            it["traffic"] = int(2 * m["FETCH_SIZE"] * 1024 + m.get("WRITE_SIZE", 0) * 1024)
        res[k] = it
    json.dump({"tree": product_tree(), "kernels": res}, open(out, "w"), indent=1)
    for k, it in res.items():
        print(k[:70], it.get("pmc_dur_us"), it.get("mfma_util"), it.get("traffic"))
        for c, v in sorted(it["counters"].items()):
            print(f"   {c:28s} {v:16.1f}")


if __name__ == "__main__":
    main()
