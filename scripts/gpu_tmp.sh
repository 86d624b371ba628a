set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t7; mkdir -p $O
bash scripts/gpu_ab.sh t7/ab base dw4 aw5 base dw4 aw5 || exit 1
timeout -k 10 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"
tail -30 $O/pytest.log | grep -E "passed|failed|FAILED|Error"
