"""Per-instance kernel timing from a rocprofv3 kernel_trace.csv: groups dispatches by
(kernel, grid, block) and prints avg duration, count, VGPRs; sorted by total time."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
filt = sys.argv[3] if len(sys.argv) > 3 else ""
g = defaultdict(list)
meta = {}
for r in rows:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    if filt and filt not in name:
        continue
    key = (name, int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) // max(1, int(r["Workgroup_Size_X"])), int(r["Workgroup_Size_X"]))
    g[key].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    meta[key] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["LDS_Block_Size"])
tot = sum(sum(v) for v in g.values())
for key, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:top]:
    name, wgs, bs = key
    print(f"{sum(v) / tot * 100:5.1f}%  n={len(v):4d}  avg {sum(v) / len(v) / 1000:8.2f}us  wg={wgs:6d}x{bs:<4d} vgpr={meta[key][0]:>3} lds={meta[key][2]:>6}  {name[:60]}")
