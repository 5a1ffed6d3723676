"""Per-launch list of one training step from a rocprofv3 kernel trace (kernel, grid, time)."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -3
ends = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
seg = rows[ends[which] + 1:ends[which + 1] + 1]
tot = 0.0
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    n = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "")
    n = re.sub(r"\(.*", "", n)
    print(f"{d:7.1f} {n[:44]:44s} {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}/"
          f"{r['Workgroup_Size_X']} v{r['VGPR_Count']}")
print(f"sum {tot:.1f} us, {len(seg)} launches")
