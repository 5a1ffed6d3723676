"""Splits a rocprofv3 kernel trace into training steps (at each adamw launch) and reports,
per step, wall time vs summed kernel time, launch count and the largest idle gaps."""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "adamw"
ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
gaps = defaultdict(list)
for a, b in zip(ends[:-1], ends[1:]):
    seg = rows[a + 1:b + 1]
    t0 = int(seg[0]["Start_Timestamp"]); t1 = int(seg[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in seg)
    gap = [int(y["Start_Timestamp"]) - int(x["End_Timestamp"]) for x, y in zip(seg[:-1], seg[1:])]
    print(f"step: wall {(t1 - t0) / 1e3:8.1f}us busy {busy / 1e3:8.1f}us n={len(seg)} "
          f"gap-sum {sum(gap) / 1e3:7.1f}us median-gap {sorted(gap)[len(gap) // 2] / 1e3:.2f}us")
