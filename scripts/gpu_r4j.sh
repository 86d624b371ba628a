#!/bin/bash
# round 4: the streamed windows as elimination + walk launches by default
# (TORJ_DEPO_STREAM=3) with the walk one segment at a time at three waves per
# SIMD -- the deposition GPU tests, then an alternating A/B against HEAD
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_deposition.py tests/test_gpu_c3.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/gpu_ab.sh r4j/ab head base head base head base || exit 1
