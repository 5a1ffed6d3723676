"""Average duration of the dominant call's kernel from a rocprofv3 kernel trace, selecting the
dispatches of that exact launch shape (kernel name + grid size), so that it can be compared with
bench.py's HIP-event `roofline.avg_launch_ms`.

    python tools/dom_trace.py <run_kernel_trace.csv> [name-substring] [grid_x]
default: dw3p_bwd_kernel<0, 16, true> with grid 3840 x 64 = [4, 32, 48^3] (3840 one-wave tiles)
"""
import csv
import json
import sys

path = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else "dw3p_bwd_kernel<0, 16, true>"
grid = int(sys.argv[3]) if len(sys.argv) > 3 else 3840 * 64
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
     for r in csv.DictReader(open(path))
     if sub in r["Kernel_Name"] and int(r["Grid_Size_X"]) == grid]
out = {"kernel": sub, "grid_x": grid, "dispatches": len(d),
       "avg_us": round(sum(d) / len(d), 3) if d else None,
       "min_us": round(min(d), 3) if d else None, "max_us": round(max(d), 3) if d else None}
print(json.dumps(out))
