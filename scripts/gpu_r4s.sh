#!/bin/bash
# round 4: alpha workgroups of 192 lanes (b192) against 128 (base) on C3, and
# the warm alpha kernel at 128 lanes (w128) against 256 (base) on C5, alternating;
# the warm GPU tests on w128
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4s
mkdir -p $O
W128=$PWD/torj.jl_amd/build/variants/libtorj_hip_w128.so
TORJ_HIP_LIB=$W128 timeout -k 10 600 python -u -m pytest tests/test_gpu_warm.py tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "warm" > $O/pytest_w128.log 2>&1 || { tail -30 $O/pytest_w128.log; exit 1; }
tail -1 $O/pytest_w128.log
bash scripts/gpu_ab.sh r4s/c3 base b192 base b192 base b192 || exit 1
BENCH_ARGS="--absorption warm_wr" bash scripts/gpu_ab.sh r4s/c5 base w128 base w128 || exit 1
