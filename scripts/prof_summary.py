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
groups = defaultdict(float)
for r in rows:
    n = r["Name"]
    if n.startswith("Cijk") or n.startswith("Custom_Cijk"):
        g = "GEMM (hipBLASLt)"
    elif "attn" in n:
        g = "attention"
    elif "norm" in n:
        g = "norm"
    elif "nccl" in n.lower() or "rccl" in n.lower():
        g = "collectives"
    else:
        g = re.sub(r"\(.*", "", n).replace("void ", "").replace("(anonymous namespace)::", "")[:40]
    groups[g] += float(r["TotalDurationNs"])
print("\n-- groups --")
for g, v in sorted(groups.items(), key=lambda x: -x[1])[:20]:
    print(f"{v/1e6/steps:9.3f} ms/step {100*v/tot:6.2f}%  {g}")
print("\n-- top kernels --")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    name = r["Name"].replace("(anonymous namespace)::", "")
    print(f"{float(r['TotalDurationNs'])/1e6/steps:8.3f} ms/step calls={int(r['Calls'])/steps:6.1f}/step "
          f"avg={float(r['AverageNs'])/1e3:8.1f}us  {name[:100]}")
