#!/bin/bash
# Tiled trajectory kernel (TORJ_TRAJ_LDS=2) vs the whole-grid LDS kernel (=1):
# its GPU tests, an alternating bench A/B, and a serialised rocprof of each
# bash scripts/gpu_tile_ab.sh OUTDIR
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -s -k "tile" > $O/pytest_tile.log 2>&1 || { tail -30 $O/pytest_tile.log; exit 1; }
grep -E "passed|failed|TORJ_TRAJ" $O/pytest_tile.log | tail -5
bash scripts/gpu_env_ab.sh $1/ab 'lds1:TORJ_TRAJ_LDS=1' 'tile:TORJ_TRAJ_LDS=2' 'lds1b:TORJ_TRAJ_LDS=1' 'tileb:TORJ_TRAJ_LDS=2' || exit 1
for v in 1 2; do
  TORJ_TRAJ_LDS=$v TORJ_SPLIT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/st$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --steps 2 > $O/st$v.log 2>&1 || exit 1
  f=$(find $O/st$v -name '*kernel_stats.csv' | head -1); grep -E "k_traj|k_alpha_pts|k_tau|k_depo" $f | cut -d, -f1-5
done
for v in 1 2; do
  TORJ_TRAJ_LDS=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/ov$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --steps 2 > $O/ov$v.log 2>&1 || exit 1
  f=$(find $O/ov$v -name '*kernel_stats.csv' | head -1); grep -E "k_traj|k_alpha_pts|k_tau|k_depo" $f | cut -d, -f1-5
done
