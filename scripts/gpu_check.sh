#!/bin/bash
# GPU tests + headline bench (+ optional extra bench args for a second line) -> gpurun_out/check/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/check
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
python tools/bench_brief.py $O/bench_c3.log
if [ -n "$1" ]; then
  timeout -k 10 400 python bench.py --no-cpu-baseline $1 > $O/bench_extra.log 2>&1 || { tail -20 $O/bench_extra.log; exit 1; }
  python tools/bench_brief.py $O/bench_extra.log
fi
