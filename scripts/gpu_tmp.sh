set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_ab.sh t12/ab base tp3 tp3ap1 base tp3 tp3ap1 || exit 1
