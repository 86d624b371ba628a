#!/bin/bash
# round 4: only the alpha / scan streams on a CU mask (TORJ_ALPHA_CUS = Y of
# the 256 CUs), the trajectory stream unmasked, alternating with no masks
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_env_ab.sh r4m/cus 'a0:TORJ_ALPHA_CUS=0' 'a224:TORJ_ALPHA_CUS=224' 'a192:TORJ_ALPHA_CUS=192' 'a160:TORJ_ALPHA_CUS=160' 'a128:TORJ_ALPHA_CUS=128' 'a240:TORJ_ALPHA_CUS=240' 'a0b:TORJ_ALPHA_CUS=0' 'a224b:TORJ_ALPHA_CUS=224' 'a192b:TORJ_ALPHA_CUS=192' 'a160b:TORJ_ALPHA_CUS=160' || exit 1
