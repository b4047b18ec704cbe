#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 --pmc counters: python scripts/pmc_table.py DIR [DIR ...] [--match SUBSTR]"""
import collections
import csv
import sys

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = sys.argv[sys.argv.index("--match") + 1] if "--match" in sys.argv else ""
if match in args:
    args.remove(match)
for d in args:
    rows = list(csv.DictReader(open(f"{d}/run_counter_collection.csv")))
    agg = collections.OrderedDict()
    for r in rows:
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if match and match not in k:
            continue
        agg.setdefault(k[:60], collections.OrderedDict()).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    print(f"== {d}")
    for k, cs in agg.items():
        print("  " + k)
        print("    " + "  ".join(f"{c}={sum(v)/len(v):.4g}" for c, v in cs.items()))
