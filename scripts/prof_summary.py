#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels, per-step time, groups."""
import csv
import re
import sys
from collections import defaultdict

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(f"{d}/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.2f} ms  ({tot/1e6/steps:.3f} ms/step over {steps:g} steps)")
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


groups = defaultdict(float)
for r in rows:
    groups[group_of(r["Name"])] += float(r["TotalDurationNs"])
print("\n-- groups --")
for g, v in sorted(groups.items(), key=lambda x: -x[1])[:20]:
    print(f"{v/1e6/steps:9.3f} ms/step {100*v/tot:6.2f}%  {g}")
print("\n-- top kernels --")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    name = short(r["Name"])
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step calls={int(r['Calls'])/steps:6.1f}/step "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us  {name[:100]}")
