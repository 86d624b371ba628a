set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_env_ab.sh t10/env 'base:' 'as2:TORJ_ALPHA_STREAMS=2' 'base2:' 'as2b:TORJ_ALPHA_STREAMS=2' || exit 1
