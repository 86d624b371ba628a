#!/bin/bash
# round 4 profile of HEAD (C3): rocprof kernel trace + PMC passes -> profiles/r04,
# an LDS pass of the trajectory kernel, and the split-ring size A/B with its HBM bytes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O/profiles
bash scripts/profile.sh prof_r4 || exit 1
python tools/prof_summary.py gpurun_out/prof_r4 $O/profiles "k_traj|k_alpha_pts|k_tau_scan|k_split_final|k_depo_stream" || exit 1
python tools/prof_summary.py gpurun_out/prof_r4 $O/profiles k_depo_tail depo_ || exit 1
(cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/$O/lds -o lds -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-api > $GRAFT_REPO_ROOT/$O/lds.log 2>&1) || { echo lds pass failed; tail -5 $O/lds.log; exit 1; }
python - <<'PY' || exit 1
import csv, glob
from collections import defaultdict
f = glob.glob("gpurun_out/r4e/lds/**/*counter_collection.csv", recursive=True)[0]
t = defaultdict(lambda: defaultdict(float)); n = defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "")
    t[k][r["Counter_Name"]] += float(r["Counter_Value"]); n[k].add(r["Dispatch_Id"])
for k, v in t.items():
    if v.get("SQ_INSTS_LDS", 0) > 0:
        print(k, len(n[k]), {c: round(x / 1e9, 3) for c, x in v.items()})
PY
bash scripts/gpu_ring_ab.sh r4e/ring || exit 1
