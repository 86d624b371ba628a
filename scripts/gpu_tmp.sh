set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t8; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -q -m gpu -k "streamed_deposition" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -3 $O/pytest.log
bash scripts/gpu_env_ab.sh t8/env 'base:' 'd5:TORJ_DEPO_STREAM=5' 'd5l1:TORJ_DEPO_STREAM=5 TORJ_DEPO_LAG=1' 'd5l3:TORJ_DEPO_STREAM=5 TORJ_DEPO_LAG=3' 'base2:' 'd5b:TORJ_DEPO_STREAM=5' 'd5l1b:TORJ_DEPO_STREAM=5 TORJ_DEPO_LAG=1' 'd5l3b:TORJ_DEPO_STREAM=5 TORJ_DEPO_LAG=3' || exit 1
