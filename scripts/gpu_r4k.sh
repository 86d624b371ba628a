#!/bin/bash
# round 4: a fixed CU partition between the trajectory stream and the alpha /
# scan streams (TORJ_TRAJ_CUS = X of the 256 CUs; 0: no masks), alternating
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r4k/cus 'c0:TORJ_TRAJ_CUS=0' 'c98:TORJ_TRAJ_CUS=98' 'c112:TORJ_TRAJ_CUS=112' 'c128:TORJ_TRAJ_CUS=128' 'c84:TORJ_TRAJ_CUS=84' 'c66:TORJ_TRAJ_CUS=66' 'c0b:TORJ_TRAJ_CUS=0' 'c98b:TORJ_TRAJ_CUS=98' 'c112b:TORJ_TRAJ_CUS=112' 'c128b:TORJ_TRAJ_CUS=128' || exit 1
