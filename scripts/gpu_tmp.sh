set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/g23; mkdir -p $O
timeout -k 10 600 bash scripts/gpu_ab.sh g23 prevsum base prevsum base || exit 1
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -k "deposition or c3 or beam" --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
