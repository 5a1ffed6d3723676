"""Turns the two rocprofv3 PMC passes of tools/pmc.sh (FETCH_SIZE, WRITE_SIZE; kernel-trace only)
into the per-call traffic record bench.py reads (profiles/<tag>_pmc_dw3_bwd.json).
FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 tallies 16-B/lane streaming reads at half);
both counters are in KiB.  Calls 3-10 of tools/pmc_dw.py's 10 calls are averaged.

    python tools/pmc_json.py <pmc out dir> <out.json>
"""
import collections
import csv
import glob
import json
import re
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from treehash import product_tree  # noqa: E402


def per_kernel(d, counter):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{d}/{counter}/**/*counter_collection.csv", recursive=True):
        rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Dispatch_Id"]))
        for r in rows:
            if r["Counter_Name"] != counter or "dw3" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
            name = re.sub(r"\(.*", "", name).replace("void ", "")
            vals[name].append(float(r["Counter_Value"]) * 1024)
    return {k: sum(v[2:10]) / len(v[2:10]) for k, v in vals.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch = per_kernel(d, "FETCH_SIZE")
    write = per_kernel(d, "WRITE_SIZE")
    ks = {k: {"fetch_bytes": int(2 * fetch.get(k, 0)), "write_bytes": int(write.get(k, 0))}
          for k in sorted(set(fetch) | set(write))}
    rec = {"call": "l3u_dw3_bwd [4,32,48^3] (accumulate=1, no IN record): 10 calls, calls 3-10 averaged",
           "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes with "
                     "--kernel-trace only (tools/pmc.sh); FETCH_SIZE doubled per MI355X_MICROARCH.md "
                     "(gfx950 reports half the bytes of 16-B/lane streaming reads); values in bytes per call",
           "kernels": ks,
           "traffic_bytes": sum(v["fetch_bytes"] + v["write_bytes"] for v in ks.values()),
           "algorithmic_bytes": 4 * 4 * 4 * 32 * 48 ** 3 + 4 * 27 * 32}
    rec["tree"] = product_tree()
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
