#!/bin/bash
# round 4: deposition windows on their own stream (TORJ_DEPO_STREAM=2) -- its
# GPU test, then alternating trace-phase A/Bs (+ more hardware queues, + the
# one-segment walk batch variant)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "streamed or serial_equals" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log
bash scripts/gpu_env_ab.sh r4b/env 's1:TORJ_DEPO_STREAM=1' 's2:TORJ_DEPO_STREAM=2' 's2q8:TORJ_DEPO_STREAM=2 GPU_MAX_HW_QUEUES=8' 's0:TORJ_DEPO_STREAM=0' 's1b:TORJ_DEPO_STREAM=1' 's2b:TORJ_DEPO_STREAM=2' 's2q8b:TORJ_DEPO_STREAM=2 GPU_MAX_HW_QUEUES=8' 's0b:TORJ_DEPO_STREAM=0' || exit 1
bash scripts/gpu_ab.sh r4b/var base w1 base w1 || exit 1
