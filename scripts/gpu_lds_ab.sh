#!/bin/bash
# A/B of the trajectory kernel's coefficient source (L2 vs LDS, TORJ_TRAJ_LDS) in
# the split pipeline: parity tests with LDS, bench lines, serial per-kernel times
# and VMEM-read counts -> gpurun_out/$1
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; mkdir -p $O
TORJ_TRAJ_LDS=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_lds.log 2>&1; tail -2 $O/pytest_lds.log
for v in 0 1; do TORJ_TRAJ_LDS=$v bash scripts/gpu_ab.sh $1/lds$v base || exit 1; done
cd /tmp && export TMPDIR=/tmp
for v in 0 1; do
  TORJ_TRAJ_LDS=$v TORJ_SPLIT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/st$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 > /dev/null 2>&1 || exit 1
  TORJ_TRAJ_LDS=$v TORJ_SPLIT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc$v -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 1 --warmup 0 > /dev/null 2>&1 || exit 1
done
echo done
