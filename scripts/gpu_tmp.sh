set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t4; mkdir -p $O
TORJ_PRIO_VERBOSE=1 timeout -k 10 120 python bench.py --no-cpu-baseline --no-host-api --steps 1 --warmup 0 2>&1 | grep "torj:" | head -5
bash scripts/gpu_env_ab.sh t4/env 'base:' 'ahi:TORJ_ALPHA_PRIO=-10' 'ahitlo:TORJ_ALPHA_PRIO=-10 TORJ_TRAJ_PRIO=10' 'ds0:TORJ_DEPO_STREAM=0' 'ds4:TORJ_DEPO_STREAM=4' 'base2:' 'ahi2:TORJ_ALPHA_PRIO=-10' 'ahitlo2:TORJ_ALPHA_PRIO=-10 TORJ_TRAJ_PRIO=10' || exit 1
bash scripts/gpu_ab.sh t4/ab base sp2 ab256 base sp2 ab256 || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_c3.py -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; echo "pytest rc=$?"
tail -30 $O/pytest.log | grep -E "passed|failed|FAILED|Error"
