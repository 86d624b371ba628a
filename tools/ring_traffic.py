#!/usr/bin/env python3
"""HBM bytes per launch of the split pipeline's trace phase for each ring block
size of scripts/gpu_ring_ab.sh (FETCH_SIZE and WRITE_SIZE in KiB, summed over
the dispatches of one timed launch; gfx950 correction of MI355X_MICROARCH.md
"HBM": FETCH_SIZE x 2), with the A/B's trace-phase times beside them.
usage: python tools/ring_traffic.py gpurun_out/<dir>  ->  <dir>/ring_traffic.json"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

KERNELS = ("k_traj", "k_alpha_pts", "k_tau_scan", "k_split_final", "k_depo_stream")


def per_launch(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        return None
    tot, marks = defaultdict(float), set()
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"]
        if "k_split_final" in name:
            marks.add(r["Dispatch_Id"])
        if any(k in name for k in KERNELS):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
    n = max(len(marks), 1)  # launches: the counted one and the timed one
    return tot[counter] * 1024.0 / n


def main(src):
    out = {}
    for mb in (1024, 256, 128, 64):
        fe = per_launch(os.path.join(src, f"pmc_{mb}_FETCH_SIZE"), "FETCH_SIZE")
        wr = per_launch(os.path.join(src, f"pmc_{mb}_WRITE_SIZE"), "WRITE_SIZE")
        ms = []
        for log in sorted(glob.glob(os.path.join(src, "ab", f"mb{mb}*.log"))):
            for line in open(log):
                if line.startswith("{"):
                    ms.append(json.loads(line)["roofline"]["kernel_ms"])
        out[f"{mb}MiB"] = {"fetch_bytes_corrected": 2 * fe if fe is not None else None,
                           "write_bytes": wr,
                           "hbm_bytes_per_launch": (2 * fe + wr) if fe is not None and wr is not None else None,
                           "trace_phase_ms": ms}
    json.dump(out, open(os.path.join(src, "ring_traffic.json"), "w"), indent=1)
    for k, v in out.items():
        print(k, {a: (round(b / 1e9, 2) if isinstance(b, float) else b) for a, b in v.items()})


if __name__ == "__main__":
    main(sys.argv[1])
