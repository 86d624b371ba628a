#!/bin/bash
# A/B of register footprints beside the tiled trajectory kernel: the streamed
# deposition's VGPR cap (ds3 / ds4), the trajectory's (t3 / t4), both (t3ds4)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TORJ_TRAJ_LDS=2
bash scripts/gpu_ab.sh $1 base ds4 ds3 t3 t4 t3ds4 base ds4 t3 t3ds4 || exit 1
bash scripts/gpu_env_ab.sh $1/env 'nostream:TORJ_DEPO_STREAM=0' 'stream:TORJ_DEPO_STREAM=1' 'nostream2:TORJ_DEPO_STREAM=0' || exit 1
