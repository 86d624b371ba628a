#!/bin/bash
# round 4: alpha waves-per-SIMD bound 5 / 3 (aw5, aw3) and 12-cell trajectory
# tiles (tc12) against the default on C3; warm alpha groups of 64 lanes (ww64)
# against 128 on C5; alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_ab.sh r4t/c3 base aw5 aw3 tc12 base aw5 aw3 tc12 || exit 1
BENCH_ARGS="--absorption warm_wr" bash scripts/gpu_ab.sh r4t/c5 base ww64 base ww64 || exit 1
