#!/usr/bin/env python3
"""Idle gaps between consecutive kernels in a rocprofv3 kernel trace (single queue view).

    python scripts/prof_gaps.py DIR [last_fraction]

Sorts dispatches by start time, keeps the last fraction of the trace (the timed steps), and reports
busy time, idle time between kernels, and the largest gaps with the kernels around them.
"""
import csv
import sys

d = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
rows = list(csv.DictReader(open(f"{d}/run_kernel_trace.csv")))
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
ev = ev[int(len(ev) * (1 - frac)):]
t0, t1 = ev[0][0], max(e[1] for e in ev)
busy, gaps, end = 0, [], ev[0][0]
for s, e, n in ev:
    if s > end:
        gaps.append((s - end, n))
    busy += max(0, e - max(s, end))
    end = max(end, e)
wall = t1 - t0
print(f"kernels {len(ev)}  wall {wall/1e6:.3f} ms  busy {busy/1e6:.3f} ms  idle {(wall-busy)/1e6:.3f} ms "
      f"({100*(wall-busy)/wall:.1f}%)  gaps>0: {len(gaps)}  mean gap {sum(g for g,_ in gaps)/max(1,len(gaps))/1e3:.2f} us")
for g, n in sorted(gaps, reverse=True)[:12]:
    print(f"  {g/1e3:8.1f} us before {n[:90]}")
