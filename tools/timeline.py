#!/usr/bin/env python3
"""Per-launch timeline of the split pipeline from a rocprofv3 kernel trace:
for one launch (the n-th k_split_final and the kernels since the previous
one), each stream's busy time, the trajectory kernels' durations and the gaps
between consecutive trajectory kernels (time the trajectory chain waited).
usage: python tools/timeline.py trace_kernel_trace.csv [launch_index]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
li = int(sys.argv[2]) if len(sys.argv) > 2 else 50
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ends = [k for k, r in enumerate(rows) if "k_split_final" in r["Kernel_Name"]]
lo, hi = ends[li - 1] + 1, ends[li]
seg = rows[lo:hi + 1]
t0 = int(seg[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in seg)
print(f"launch {li}: {len(seg)} dispatches, span {(t1 - t0) / 1e6:.2f} ms")
busy = defaultdict(float)
kinds = defaultdict(list)
for r in seg:
    name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    kinds[name].append((s, e))
    busy[name] += (e - s) / 1e6
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {k:24s} {len(kinds[k]):4d} x  sum {v:8.2f} ms  mean {v / len(kinds[k]):.3f} ms")
tr = sorted(kinds.get("k_traj_cell", []))
gaps = [(tr[k + 1][0] - tr[k][1]) / 1e6 for k in range(len(tr) - 1)]
if gaps:
    print(f"  trajectory chain: first start +{(tr[0][0] - t0) / 1e6:.3f} ms, last end +{(tr[-1][1] - t0) / 1e6:.2f} ms, "
          f"gaps sum {sum(gaps):.2f} ms (max {max(gaps):.3f})")
    print("  per block (start offset ms, duration ms):", " ".join(f"{(s - t0) / 1e6:.1f}/{(e - s) / 1e6:.2f}" for s, e in tr[:40]))
al = sorted(kinds.get("k_alpha_pts", []) + kinds.get("k_alpha_warm_pts", []))
if al:
    print("  alpha per block:", " ".join(f"{(s - t0) / 1e6:.1f}/{(e - s) / 1e6:.2f}" for s, e in al[:40]))
sc = sorted(kinds.get("k_tau_scan", []))
if sc:
    print("  scan per block:", " ".join(f"{(s - t0) / 1e6:.1f}/{(e - s) / 1e6:.2f}" for s, e in sc[:40]))
