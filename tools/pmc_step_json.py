"""Per-launch HBM traffic of one eager training step from tools/pmc_step.sh's two passes:
FETCH_SIZE (x2, the gfx950 correction of MI355X_MICROARCH.md) + WRITE_SIZE, KiB -> bytes.
Steps end at each adamw launch; the last complete step is reported, in launch order.

    python tools/pmc_step_json.py <pmc out dir> <out.json>
"""
import csv
import json
import re
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from treehash import product_tree  # noqa: E402


def launches(d, counter):
    rows = list(csv.DictReader(open(f"{d}/{counter}/run_counter_collection.csv")))
    rows = [r for r in rows if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    out = []
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).replace("void ", "")
        out.append((name, int(r["Grid_Size"]) if "Grid_Size" in r else 0, float(r["Counter_Value"]) * 1024))
    return out


def last_step(seq):
    ends = [i for i, (n, _, _) in enumerate(seq) if "adamw" in n]
    a, b = ends[-2], ends[-1]
    return seq[a + 1:b + 1]


def main():
    d, out = sys.argv[1], sys.argv[2]
    f = last_step(launches(d, "FETCH_SIZE"))
    w = last_step(launches(d, "WRITE_SIZE"))
    assert [x[0] for x in f] == [x[0] for x in w], "passes disagree on the launch sequence"
    items = [{"kernel": a[0], "fetch_x2": 2 * a[2], "write": b[2], "traffic": 2 * a[2] + b[2]}
             for a, b in zip(f, w)]
    tot = sum(i["traffic"] for i in items)
    rec = {"what": "HBM bytes per launch of one eager bs-4 48^3 training step (FETCH_SIZE x2 + "
                   "WRITE_SIZE, separate rocprofv3 passes)", "launches": len(items),
           "step_traffic_bytes": tot, "items": items}
    rec["tree"] = product_tree()
    json.dump(rec, open(out, "w"), indent=1)
    print(f"{len(items)} launches, {tot / 1e9:.3f} GB per step")
    for i in sorted(items, key=lambda i: -i["traffic"])[:25]:
        print(f"{i['traffic'] / 1e6:9.1f} MB  (fetch {i['fetch_x2'] / 1e6:8.1f}, write {i['write'] / 1e6:8.1f})  {i['kernel'][:60]}")


if __name__ == "__main__":
    main()
