#!/usr/bin/env python
"""Summarise rocprofv3 CSV output: per-kernel time table + per-kernel PMC averages."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
stats = glob.glob(os.path.join(out, "prof", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    rows = list(csv.DictReader(open(stats[0])))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"== kernel time ({tot/1e6:.1f} ms total)")
    for r in rows[:30]:
        print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {100*float(r["TotalDurationNs"])/tot:5.1f}% '
              f'n={r["Calls"]:>5} avg={float(r["AverageNs"])/1e3:8.1f}us {r["Name"][:90]}')
for d in ("pmcA", "pmcB"):
    files = glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(files[0])):
        name = r.get("Kernel_Name", r.get("Kernel-Name", "?"))[:60]
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"== {d}")
    for k, cs in acc.items():
        if "fa_" not in k and "norm" not in k:
            continue
        print(k, {c: round(sum(v) / len(v)) for c, v in cs.items()})
