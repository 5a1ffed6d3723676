"""Summary of tools/icache_probe.py's kernel trace: the probe kernel's mean duration by pattern
(A: after a streaming copy; B: after itself, same buffers; C: after itself on other buffers,
which follows the copy).   python tools/icache_summary.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in rows]
probe = [i for i, (n, _) in enumerate(ks) if "dwv_fwd" in n or "dw3" in n]
# patterns in order: A = probe after a copy with no probe just before the copy's predecessor...
# classify each probe launch by its predecessor and the predecessor's predecessor
cls = {"after copy": [], "after probe, prev-prev copy": [], "after probe, prev-prev probe": []}
for i in probe:
    p = ks[i - 1][0] if i > 0 else ""
    pp = ks[i - 2][0] if i > 1 else ""
    if "dwv" not in p and "dw3" not in p:
        cls["after copy"].append(ks[i][1])
    elif "dwv" not in pp and "dw3" not in pp:
        cls["after probe, prev-prev copy"].append(ks[i][1])
    else:
        cls["after probe, prev-prev probe"].append(ks[i][1])
for k, v in cls.items():
    if v:
        v = sorted(v)[len(v) // 10: len(v) - len(v) // 10 or None]
        print(f"{k:32s} n={len(v):4d} mean {sum(v) / len(v):6.2f} us  min {min(v):6.2f}  max {max(v):6.2f}")
