#!/bin/bash
# round 4: alpha grid order with the (step, stage) index fastest (variant jsf)
# against ray groups fastest (base), alternating; C3 sampled parity on jsf
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4v
mkdir -p $O
TORJ_HIP_LIB=$PWD/torj.jl_amd/build/variants/libtorj_hip_jsf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "sampled_parity" > $O/pytest_jsf.log 2>&1 || { tail -30 $O/pytest_jsf.log; exit 1; }
tail -1 $O/pytest_jsf.log
bash scripts/gpu_ab.sh r4v/ab base jsf base jsf base jsf || exit 1
