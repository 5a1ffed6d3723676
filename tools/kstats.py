"""Summarise a rocprofv3 kernel_stats.csv: share, calls/step, avg us per kernel."""
import csv
import sys

path = sys.argv[1]
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0]
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}%  {int(r['Calls']) / steps:7.1f}/step  "
          f"avg {float(r['AverageNs']) / 1000:8.2f}us  {name[:80]}")
print(f"total {tot / 1e6:.2f} ms = {tot / 1e6 / steps:.3f} ms/step over {steps} steps")
