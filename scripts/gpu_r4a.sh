#!/bin/bash
# round 4, first call: the C5 fan-scale GPU test, the tiled trajectory tests,
# and the register-cap A/B beside the tiled trajectory kernel
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_c5.py tests/test_gpu_split.py -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider -k "c5 or tile or cold_edge" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed|C5 fan|iwarm 1" $O/pytest.log
bash scripts/gpu_ds_ab.sh r4a/ds || exit 1
