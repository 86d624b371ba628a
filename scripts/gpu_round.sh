#!/bin/bash
# One GPU call: GPU tests, profile of the headline bench, default bench (with
# the CPU baseline) -> gpurun_out/round/
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/round
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/round/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/round/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/round/pytest_gpu.log
bash scripts/profile.sh prof_round || exit 1
python tools/prof_summary.py gpurun_out/prof_round profiles/${ROUND:-r01} k_trace || exit 1
cp profiles/${ROUND:-r01}/traffic.json profiles/${ROUND:-r01}/pmc_summary.json profiles/${ROUND:-r01}/kernel_stats.csv gpurun_out/round/
timeout -k 10 600 python bench.py > gpurun_out/round/bench.log 2>&1 || { tail -20 gpurun_out/round/bench.log; exit 1; }
grep '^{' gpurun_out/round/bench.log
