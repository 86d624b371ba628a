#!/bin/bash
# first bring-up on the GPU box: smoke, a small bench, then the headline bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "gfx|Marketing" > gpurun_out/gpuinfo.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log | tail -30; exit 1; }
tail -3 gpurun_out/smoke.log
timeout -k 10 300 python bench.py --n-rings 20 --min-az 11 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1 || { echo "small bench failed"; tail -30 gpurun_out/bench_small.log; exit 1; }
tail -2 gpurun_out/bench_small.log
timeout -k 10 400 python bench.py --steps 2 --warmup 1 --cpu-seconds 10 > gpurun_out/bench_full.log 2>&1 || { echo "full bench failed"; tail -30 gpurun_out/bench_full.log; exit 1; }
tail -2 gpurun_out/bench_full.log
