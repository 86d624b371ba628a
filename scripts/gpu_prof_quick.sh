#!/bin/bash
# fp64 issue-rate microbenchmark + PMC pass of the headline kernel -> gpurun_out/pq/
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/pq
timeout -k 10 120 ./tools/fp64_peak > gpurun_out/pq/fp64_peak.txt 2>&1 || { cat gpurun_out/pq/fp64_peak.txt; exit 1; }
cat gpurun_out/pq/fp64_peak.txt
bash scripts/profile.sh pq_prof || exit 1
python tools/prof_summary.py gpurun_out/pq_prof gpurun_out/pq k_trace
