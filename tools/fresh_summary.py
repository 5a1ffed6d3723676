"""Summary of tools/fresh_probe.py's kernel trace: the consumer's (dw3 / dwv) mean duration by
what ran just before it.   python tools/fresh_summary.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3,
       int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
cons = lambda n: "dwv_" in n or "dw3" in n  # noqa: E731
cls = {"F: after its producer": [], "O: producer one launch earlier": [], "W: after itself": []}
gaps = {k: [] for k in cls}
for i, (n, us, t0, _) in enumerate(ks):
    if not cons(n) or i < 2:
        continue
    p, pp = ks[i - 1][0], ks[i - 2][0]
    if cons(p):
        k = "W: after itself"
    elif cons(pp) or "pw_fwd" not in pp:
        k = "F: after its producer"
    else:
        k = "O: producer one launch earlier"
    cls[k].append(us)
    gaps[k].append((t0 - ks[i - 1][3]) / 1e3)
for k, v in cls.items():
    if v:
        v = sorted(v)[len(v) // 10: len(v) - len(v) // 10 or None]
        g = sorted(gaps[k])[len(gaps[k]) // 2]
        print(f"{k:32s} n={len(v):4d} mean {sum(v) / len(v):6.2f} us  min {min(v):6.2f}  gap(median) {g:5.2f} us")
