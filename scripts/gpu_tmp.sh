set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g9; mkdir -p $O
BENCH_ARGS="--absorption warm_wr" timeout -k 10 900 bash scripts/gpu_ab.sh g9 side1 base side1 base || exit 1
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "warm or c5 or deferred" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
