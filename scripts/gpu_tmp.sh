set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
rm -rf gpurun_out/round gpurun_out/prof_c3 gpurun_out/prof_c5
ROUND=r05 bash scripts/gpu_round.sh A || exit 1
ROUND=r05 bash scripts/gpu_round.sh B || exit 1
