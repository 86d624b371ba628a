#!/bin/bash
# round 4: the streamed deposition's cost -- windows as one
# kernel (TORJ_DEPO_STREAM=1, default), as elimination + walk launches (3), none
# (0); the walk at one segment per batch and four waves per SIMD (variants wc1,
# wc1w4, with TORJ_DEPO_STREAM=3); then the split-ring size A/B with its HBM
# bytes
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4i
mkdir -p $O
bash scripts/gpu_env_ab.sh r4i/depo 's1:TORJ_DEPO_STREAM=1' 's3:TORJ_DEPO_STREAM=3' 's0:TORJ_DEPO_STREAM=0' 's1b:TORJ_DEPO_STREAM=1' 's3b:TORJ_DEPO_STREAM=3' 's0b:TORJ_DEPO_STREAM=0' || exit 1
TORJ_DEPO_STREAM=3 bash scripts/gpu_ab.sh r4i/walk base wc1 wc1w4 base wc1 wc1w4 || exit 1
bash scripts/gpu_ring_ab.sh r4i/ring || exit 1
