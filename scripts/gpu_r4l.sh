#!/bin/bash
# round 4: CU partition between the trajectory stream and the alpha / scan
# streams with the tiled trajectory kernel (TORJ_TRAJ_LDS=2: one-wave
# workgroups, no one-workgroup-per-CU LDS cap), alternating with the default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r4l/cus 'c0:TORJ_TRAJ_CUS=0' 't0:TORJ_TRAJ_LDS=2 TORJ_TRAJ_CUS=0' 't96:TORJ_TRAJ_LDS=2 TORJ_TRAJ_CUS=96' 't128:TORJ_TRAJ_LDS=2 TORJ_TRAJ_CUS=128' 't80:TORJ_TRAJ_LDS=2 TORJ_TRAJ_CUS=80' 't112:TORJ_TRAJ_LDS=2 TORJ_TRAJ_CUS=112' 't64:TORJ_TRAJ_LDS=2 TORJ_TRAJ_CUS=64' 'c96:TORJ_TRAJ_CUS=96' 'c0b:TORJ_TRAJ_CUS=0' 't96b:TORJ_TRAJ_LDS=2 TORJ_TRAJ_CUS=96' || exit 1
