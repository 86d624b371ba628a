#!/usr/bin/env python3
"""Per-launch kernel milliseconds from a rocprofv3 --stats kernel_stats.csv:
python tools/kstats.py FILE [FILE...]  (launches = calls of k_split_final)"""
import csv
import sys

for f in sys.argv[1:]:
    rows = list(csv.DictReader(open(f)))
    nl = sum(int(r["Calls"]) for r in rows if "k_split_final" in r["Name"]) or 1
    print(f"{f}: {nl} launches")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"]) / 1e6 / nl
        if t >= 0.01:
            print(f"  {t:9.3f} ms/launch  {int(r['Calls']) / nl:7.1f} calls  {r['Name'][:70]}")
