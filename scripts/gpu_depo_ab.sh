#!/bin/bash
# deposition GPU tests, then A/B of variants
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ab
timeout -k 10 600 python -u -m pytest tests/test_gpu_deposition.py tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
bash scripts/gpu_ab.sh "$@"
