#!/bin/bash
# round 4: alpha workgroup size (TORJ_ALPHA_BLOCK 256 default, variants 64 and
# 128: one- and two-wave groups that fit beside the trajectory waves SIMD by
# SIMD) -- split-path GPU tests on b64, alternating A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4r
mkdir -p $O
B64=$PWD/torj.jl_amd/build/variants/libtorj_hip_b64.so
TORJ_HIP_LIB=$B64 timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_b64.log 2>&1 || { tail -30 $O/pytest_b64.log; exit 1; }
tail -1 $O/pytest_b64.log
bash scripts/gpu_ab.sh r4r/ab base b64 b128 q128 base b64 b128 q128 base b64 b128 q128 || exit 1
