#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels, per-step time, groups.

    prof_summary.py DIR STEPS              all kernels of the run (run_kernel_stats.csv) / STEPS
    prof_summary.py DIR --steady [ACCUM]   steady state only, from run_kernel_trace.csv: whole
                                           accumulation windows between loss-kernel launches (one
                                           per micro-step) after the warm-up, per micro-step, plus
                                           GPU busy time vs wall time (launch gaps)
"""
import csv
import re
import sys
from collections import defaultdict

GROUPS = [   # (group, name test) -- first match wins; every kernel lands in a named group
    ("GEMM (hipBLASLt)", lambda n: n.startswith("Cijk") or n.startswith("Custom_Cijk")),
    ("GEMM (dltb MFMA)", lambda n: n.startswith("gemm_")),
    ("attention", lambda n: n.startswith("attn_")),
    ("norm", lambda n: n.startswith("norm_")),
    ("bias/norm column sums", lambda n: n.startswith("colpart") or n.startswith("colreduce")),
    ("elementwise (gelu/swiglu/rope/dropout/scale)",
     lambda n: n.split("_")[0] in ("gelu", "swiglu", "rope", "dropout", "scale", "f32")),
    ("optimizer (adamw/grad-norm/clip)", lambda n: n.split("_")[0] in ("adamw", "sumsq", "clip", "amp")),
    ("loss (xent)", lambda n: n.startswith("xent")),
    ("embedding", lambda n: n.startswith("embed")),
    ("weight transposes", lambda n: n.startswith("transpose")),
    ("collectives (RCCL)", lambda n: "nccl" in n.lower() or "rccl" in n.lower()),
    ("torch elementwise (fill/copy/rng/index)", lambda n: n.startswith("at::")),
    ("runtime copies/fills", lambda n: n.startswith("__amd_rocclr")),
]


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.strip()


def group_of(n):
    sn = short(n)
    for g, test in GROUPS:
        if test(sn):
            return g
    return "other: " + re.sub(r"[<(].*", "", sn)[:40]


def report(rows, steps, tot):
    groups = defaultdict(float)
    for r in rows:
        groups[group_of(r["Name"])] += float(r["TotalDurationNs"])
    print("\n-- groups --")
    for g, v in sorted(groups.items(), key=lambda x: -x[1])[:20]:
        print(f"{v/1e6/steps:9.3f} ms/step {100*v/tot:6.2f}%  {g}")
    print("\n-- top kernels --")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
        name = short(r["Name"])
        print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step calls={int(r['Calls'])/steps:6.1f}/step "
              f"avg={float(r['AverageNs'])/1e3:8.1f}us  {name[:100]}")


def steady(d, marker="xent_kernel", accum=4, skip=4):
    """Kernels between two launches of ``marker`` (once per micro-step: the loss kernel) that are a
    whole number of accumulation windows apart, the first at least ``skip`` micro-steps in."""
    tr = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
    ev = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in tr))
    marks = [i for i, e in enumerate(ev) if short(e[2]).startswith(marker)]
    k2 = len(marks) - 1
    windows = (k2 - skip) // accum
    if windows < 1:
        raise SystemExit(f"need > {skip + accum} launches of {marker}, found {len(marks)}")
    k1 = k2 - windows * accum
    lo, hi = marks[k1], marks[k2]
    sel = ev[lo:hi]
    steps = windows * accum
    t0, t1 = ev[lo][0], ev[hi][0]
    busy, cur_s, cur_e = 0, None, None          # union of kernel intervals (concurrent kernels count once)
    for s_, e_, _ in sel:
        if cur_e is None or s_ > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s_, e_
        else:
            cur_e = max(cur_e, e_)
    if cur_e is not None:
        busy += cur_e - cur_s
    agg = defaultdict(lambda: [0, 0])
    for s_, e_, n in sel:
        agg[n][0] += e_ - s_
        agg[n][1] += 1
    rows = [{"Name": n, "TotalDurationNs": v[0], "Calls": v[1], "AverageNs": v[0] / v[1]} for n, v in agg.items()]
    tot = sum(v[0] for v in agg.values())
    wall = t1 - t0
    print(f"steady state: {windows} accumulation window(s) = {steps} micro-steps ({marker} launches {k1}..{k2})")
    print(f"wall {wall/1e6/steps:.3f} ms/step, GPU busy {busy/1e6/steps:.3f} ms/step ({100*busy/wall:.1f}%), "
          f"kernel time {tot/1e6/steps:.3f} ms/step, {len(sel)/steps:.0f} launches/step")
    report(rows, steps, tot)


if __name__ == "__main__":
    d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    if len(sys.argv) > 2 and sys.argv[2] == "--steady":
        steady(d, accum=int(sys.argv[3]) if len(sys.argv) > 3 else 4)
    else:
        steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
        rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
        tot = sum(float(r["TotalDurationNs"]) for r in rows)
        print(f"total kernel time {tot/1e6:.2f} ms  ({tot/1e6/steps:.3f} ms/step over {steps:g} steps)")
        report(rows, steps, tot)
