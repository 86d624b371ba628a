set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash scripts/gpu_env_ab.sh t16/env 'base:' 'old:TORJ_SPLIT_MB=1024 TORJ_SPLIT_LAST=0' 'base2:' 'old2:TORJ_SPLIT_MB=1024 TORJ_SPLIT_LAST=0' || exit 1
rm -rf gpurun_out/round gpurun_out/prof_c3 gpurun_out/prof_c5
ROUND=r05 bash scripts/gpu_round.sh A || exit 1
ROUND=r05 bash scripts/gpu_round.sh B || exit 1
