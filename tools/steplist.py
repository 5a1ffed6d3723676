"""Per-launch list of a training step from a rocprofv3 kernel trace: kernel, grid and the
duration averaged over all complete steps in the trace (steps end at each adamw launch)."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
steps = [rows[a + 1:b + 1] for a, b in zip(ends[:-1], ends[1:])]
n = len(steps[-1])
steps = [s for s in steps if len(s) == n][1:]          # same launch sequence; drop the first
tot = 0.0
for i in range(n):
    r = steps[-1][i]
    d = sum(int(s[i]["End_Timestamp"]) - int(s[i]["Start_Timestamp"]) for s in steps) / len(steps) / 1e3
    tot += d
    name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", ""))
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", name)   # bf16 instantiations stay mangled
    if m:
        name = name[m.end():m.end() + int(m.group(1))] + "<bf16 ...>"
    print(f"{d:7.1f} {name[:44]:44s} {r['Grid_Size_X']}x{r['Grid_Size_Y']}x{r['Grid_Size_Z']}/"
          f"{r['Workgroup_Size_X']} v{r['VGPR_Count']}")
print(f"sum {tot:.1f} us, {n} launches, mean of {len(steps)} steps")
