"""In-step rooflines of the depthwise, GEMM, gradient-reduction, InstanceNorm / block-tail ("norm") and
out_conv + loss ("io") families: the rocprofv3 kernel trace of the
graph-replayed training step (tools/profile.sh) aligned launch by launch with the C-ABI calls
of the same step (bench.py --dump-calls: name, family, label, algorithmic bytes).

Every kernel's duration is its mean over the complete steps of the trace (steps end at each AdamW
launch, as tools/steplist.py); kernels that are not C-ABI launches (the runtime's batch copy) are
dropped before the alignment, which must then match one kernel per call.

    python tools/instep.py <kernel_trace.csv> <calls.json> <out.json> [commit] [workload]
"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from treehash import product_tree  # noqa: E402

PEAK = 8000.0


def kernel_name(raw):
    """Readable kernel name; rocprofv3 leaves the bf16 (DF16b) instantiations mangled: keep their
    identifier and mark them <bf16 ...>."""
    n = re.sub(r"\(.*", "", raw.replace("void ", "").replace("(anonymous namespace)::", ""))
    m = re.match(r"_ZN12_GLOBAL__N_1(\d+)", n)
    if m:
        ln = int(m.group(1))
        n = n[m.end():m.end() + ln] + "<bf16 ...>"
    return n


def step_kernels(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
    steps = [rows[a + 1:b + 1] for a, b in zip(ends[:-1], ends[1:])]
    n = len(steps[-1])
    steps = [s for s in steps if len(s) == n][1:]
    out = []
    for i in range(n):
        name = kernel_name(steps[-1][i]["Kernel_Name"])
        us = sum(int(s[i]["End_Timestamp"]) - int(s[i]["Start_Timestamp"]) for s in steps) / len(steps) / 1e3
        out.append((name, us))
    return out, len(steps)


# the kernels a C-ABI call can start with (a call may launch more: e.g. l3u_convt_bwd's weight
# gradient pw_bwd_weight after its data gradient pw_fwd_ks); a kernel that cannot start the next
# call belongs to the previous one
FIRST = {
    "l3u_front_fwd": ("front_fwd",), "l3u_dwpw_fwd": ("dwpw_fwd",),
    "l3u_norm_act_pool_fwd": ("norm_act_pool_fwd",), "l3u_norm_act_fwd": ("norm_act_fwd",),
    "l3u_dw3_fwd": ("dw3", "dwv_"), "l3u_pw_fwd": ("pw_fwd",), "l3u_pw_fwd2": ("pw_fwd",),
    "l3u_convt_fwd": ("pw_fwd",), "l3u_outconv_fwd": ("outconv_fwd",),
    "l3u_norm_act_bwd": ("norm_act_bwd",), "l3u_pw_bwd": ("pw_bwd",), "l3u_dw3_bwd": ("dw3", "dwv_"),
    "l3u_convt_bwd": ("pw_fwd", "convt"), "l3u_convt_bwd_fused": ("pw_bwd_wide", "convt"),
    "l3u_maxpool2_fwd": ("maxpool",), "l3u_maxpool2_bwd": ("maxpool",),
    "l3u_reduce_segments": ("reduce_segments",), "l3u_adamw": ("adamw",),
}


def first_ok(kernel, call):
    base = call[:-5] if call.endswith("_bf16") else call
    for k in sorted(FIRST, key=len, reverse=True):
        if base.startswith(k):
            return kernel.startswith(FIRST[k])
    return True


def align(ks, calls):
    """[(call index, kernel name, us)]: kernels in launch order, each assigned to its call."""
    out, j = [], 0
    for kname, us in ks:
        if j < len(calls) and first_ok(kname, calls[j]["name"]):
            out.append((j, kname, us))
            j += 1
        elif j > 0:
            out.append((j - 1, kname, us))
        else:
            raise SystemExit(f"kernel {kname} precedes every call")
    if j != len(calls):
        raise SystemExit(f"aligned {j} of {len(calls)} calls")
    return out


def main():
    trace, calls_path, out_path = sys.argv[1:4]
    commit = sys.argv[4] if len(sys.argv) > 4 else None
    workload = sys.argv[5] if len(sys.argv) > 5 else None
    ks, nsteps = step_kernels(trace)
    ks = [k for k in ks if not k[0].startswith("__amd_rocclr")]
    calls = json.load(open(calls_path))
    per_call = {}
    for j, kname, us in align(ks, calls):
        k0, u0 = per_call.get(j, ("", 0.0))
        per_call[j] = (k0 + (" + " if k0 else "") + kname, u0 + us)
    fam = {"dw": [], "gemm": [], "reduce": [], "norm": [], "io": []}
    for j, c in enumerate(calls):
        if c["family"] is None:
            continue
        kname, us = per_call[j]
        ach = c["bytes"] / (us * 1e-6) / 1e9
        fam[c["family"]].append({"call": c["label"], "kernel": kname, "us": round(us, 2),
                                 "bytes": c["bytes"], "achieved": round(ach, 1),
                                 "frac": round(ach / PEAK, 4)})
    rec = {"what": "in-step durations (rocprofv3 kernel trace of the graph-replayed step, mean over "
                   f"{nsteps} steps) against the calls' algorithmic bytes",
           "commit": commit, "tree": product_tree(), "workload": workload,
           "step_kernel_us": round(sum(u for _, u in ks), 1), "launches": len(ks),
           "calls": len(calls)}
    for f, rows in fam.items():
        tb = sum(r["bytes"] for r in rows)
        tt = sum(r["us"] for r in rows) * 1e-6
        if not rows:
            continue
        rec[f] = {"launches": len(rows), "bytes": tb, "us": round(tt * 1e6, 1),
                  "achieved": round(tb / tt / 1e9, 1), "frac": round(tb / tt / 1e9 / PEAK, 4),
                  "calls": rows}
    # the share of the step's kernel time the families' byte models account for
    cov = sum(rec[f]["us"] for f in fam if f in rec)
    rec["coverage"] = {"family_us": round(cov, 1), "frac_of_step": round(cov / rec["step_kernel_us"], 4)}
    rec["under_10us"] = {"launches": sum(1 for _, u in ks if u < 10.0),
                         "us": round(sum(u for _, u in ks if u < 10.0), 1)}
    json.dump(rec, open(out_path, "w"), indent=1)
    print(f"{out_path}: step {rec['step_kernel_us']} us / {len(ks)} launches; dw {rec['dw']['frac']} "
          f"gemm {rec['gemm']['frac']}; <10us {rec['under_10us']}")


if __name__ == "__main__":
    main()
