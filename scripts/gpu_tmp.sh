set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
ROUND=r05 bash scripts/gpu_round.sh B || exit 1
