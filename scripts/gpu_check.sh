#!/bin/bash
# One GPU call during development: the GPU suite (verbose, per-test timeout),
# then the default bench line and the N-replica library-path rehearsal on one
# device -> gpurun_out/check/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/check
mkdir -p $O
K=${PYTEST_K:-}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu ${K:+-k "$K"} --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log | cut -c1-600
TORJ_BEAM_SAME_DEVICE=1 timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 1 > $O/bench_lib2.log 2>&1 || { tail -20 $O/bench_lib2.log; exit 1; }
grep '^{' $O/bench_lib2.log | cut -c1-1500
