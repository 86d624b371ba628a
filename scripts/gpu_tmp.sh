set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g5; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "warm or c5 or nan_alpha or deferred" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
ROUND=r05 timeout -k 10 700 bash scripts/gpu_prof.sh c5 || exit 1
