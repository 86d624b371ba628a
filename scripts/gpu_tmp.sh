set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 bash scripts/gpu_ab.sh g13 base tw3 aw6 base tw3 aw6 || exit 1
