#!/usr/bin/env python3
"""Summarise a scripts/profile.sh output directory into profiles/<round>/.

usage: python tools/prof_summary.py gpurun_out/<tag> profiles/r01 [kernel-substring] [prefix]
       kernel-substring with '|' (e.g. "k_traj|k_alpha|k_pend|k_tau_scan|k_split_final"): the
       split RK4 pipeline -- counters summed per launch over all its kernels
       (the workload is read from the JSON line of <tag>/trace.log; prefix, e.g.
       "c5_", names the outputs of a non-headline workload)

Writes
  kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  pmc_summary.json   per-dispatch averages of every PMC counter of the hot kernel
  traffic.json       HBM traffic per launch of the hot kernel, from FETCH_SIZE /
                     WRITE_SIZE (KiB) with the gfx950 correction of
                     MI355X_MICROARCH.md "HBM": FETCH_SIZE x 2; plus the executed
                     fp64 FLOPs per launch from the SQ_INSTS_VALU_*_F64 counters
                     (wave instructions x 64 lanes, FMA x 2: masked lanes count)
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict


def workload(src):
    try:
        for line in open(os.path.join(src, "trace.log")):
            if line.startswith("{"):
                d = json.loads(line)
                c = d["config"]
                return {"rays": c["rays_per_gpu"], "rk4_steps": c["rk4_steps"],
                        "n_psi": c.get("n_psi"), "traj_stride": c.get("traj_stride"),
                        "absorption": c.get("absorption", "albajar"),
                        "build_id": c.get("build_id"), "torj_env": c.get("torj_env", {}),
                        "kernel_ms_bench": d["roofline"]["kernel_ms"]}
    except (OSError, ValueError, KeyError):
        pass
    return {}


def pipeline(src, dst, pre, keys, marker):
    """The split RK4 path: counters summed over all dispatches of the pipeline's
    kernels (`keys`, '|'-separated substrings) and divided by the number of
    launches (dispatches of `marker`, one per launch) -> per-launch totals."""
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    if stats:
        shutil.copy(stats[0], os.path.join(dst, pre + "kernel_stats.csv"))
    tot = defaultdict(float)
    launches = defaultdict(set)
    per_kernel = defaultdict(lambda: defaultdict(float))
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if marker in name:
                launches[f].add(r["Dispatch_Id"])
            k = next((k for k in keys if k in name), None)
            if k is None:
                continue
            tot[(f, r["Counter_Name"])] += float(r["Counter_Value"])
            per_kernel[k][(f, r["Counter_Name"])] += float(r["Counter_Value"])
    pmc, kern = {}, defaultdict(dict)
    for (f, c), v in tot.items():
        nl = max(len(launches[f]), 1)
        pmc[c] = v / nl
        for k in keys:
            kern[k][c] = per_kernel[k].get((f, c), 0.0) / nl
    out = {"kernel": "|".join(keys), "per": "launch (sum over the pipeline's dispatches)",
           "launches_per_pass": {os.path.basename(os.path.dirname(f)): len(v) for f, v in launches.items()},
           "avg": dict(sorted(pmc.items())), "by_kernel": kern}
    json.dump(out, open(os.path.join(dst, pre + "pmc_summary.json"), "w"), indent=1)
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch = 2.0 * pmc["FETCH_SIZE"] * 1024.0
        write = pmc["WRITE_SIZE"] * 1024.0
        tr = {"kernel": "|".join(keys), "fetch_bytes": fetch, "write_bytes": write,
              "traffic_bytes": fetch + write,
              "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, summed over "
                        "the pipeline's dispatches per launch; FETCH_SIZE x2 (gfx950), KiB -> bytes",
              "source": os.path.basename(os.path.normpath(src)), "workload": workload(src)}
        f64 = [pmc.get("SQ_INSTS_VALU_" + k + "_F64") for k in ("FMA", "ADD", "MUL", "TRANS")]
        if all(v is not None for v in f64):
            tr["fp64_flops_executed"] = 64.0 * (2.0 * f64[0] + f64[1] + f64[2] + f64[3])
        json.dump(tr, open(os.path.join(dst, pre + "traffic.json"), "w"), indent=1)
        print(json.dumps(tr))


def main():
    src, dst = sys.argv[1], sys.argv[2]
    key = sys.argv[3] if len(sys.argv) > 3 else "k_trace"
    pre = sys.argv[4] if len(sys.argv) > 4 else ""
    if "|" in key:  # a pipeline of kernels: per-launch sums, launches counted by k_split_final
        os.makedirs(dst, exist_ok=True)
        return pipeline(src, dst, pre, key.split("|"), "k_split_final")
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    hot = None
    if stats:
        shutil.copy(stats[0], os.path.join(dst, pre + "kernel_stats.csv"))
        for r in csv.DictReader(open(stats[0])):
            if key in r["Name"] and (hot is None or float(r["TotalDurationNs"]) > hot[2]):
                hot = (r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]))
    vals = defaultdict(list)
    meta = {}
    for f in sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            if key not in r["Kernel_Name"]:
                continue
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            meta = {k: r[k] for k in ("Kernel_Name", "Grid_Size", "Workgroup_Size", "Scratch_Size",
                                      "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "LDS_Block_Size")}
    pmc = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
    out = {"kernel": meta, "dispatches_per_counter": {k: len(v) for k, v in vals.items()}, "avg": pmc}
    if hot:
        out["kernel_stats"] = {"name": hot[0], "calls": hot[1], "avg_ns": hot[3]}
    json.dump(out, open(os.path.join(dst, pre + "pmc_summary.json"), "w"), indent=1)
    if "FETCH_SIZE" in pmc and "WRITE_SIZE" in pmc:
        fetch = 2.0 * pmc["FETCH_SIZE"] * 1024.0  # KiB, half-counted on gfx950
        write = pmc["WRITE_SIZE"] * 1024.0
        tr = {"kernel": meta.get("Kernel_Name"), "fetch_bytes": fetch, "write_bytes": write,
              "traffic_bytes": fetch + write,
              "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes, per-dispatch "
                        "average; FETCH_SIZE x2 (gfx950), KiB -> bytes",
              "source": os.path.basename(os.path.normpath(src)), "workload": workload(src)}
        f64 = [pmc.get("SQ_INSTS_VALU_" + k + "_F64") for k in ("FMA", "ADD", "MUL", "TRANS")]
        if all(v is not None for v in f64):
            tr["fp64_flops_executed"] = 64.0 * (2.0 * f64[0] + f64[1] + f64[2] + f64[3])
        json.dump(tr, open(os.path.join(dst, pre + "traffic.json"), "w"), indent=1)
        print(json.dumps(tr))
    if hot:
        print(f"{hot[0]}: {hot[1]} calls, avg {hot[3] / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
