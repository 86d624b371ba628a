#!/bin/bash
# round 4: the cell-tiled trajectory kernel (TORJ_TRAJ_LDS=3, per-cell power
# form) -- its GPU tests, an alternating A/B against the whole-grid LDS kernel
# (=1, the default) and the node tile (=2), and a bench line with parity on it
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4n
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider -k "tile" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed|vs [23]:" $O/pytest.log
bash scripts/gpu_env_ab.sh r4n/ab 'l1:TORJ_TRAJ_LDS=1' 'l3:TORJ_TRAJ_LDS=3' 'l2:TORJ_TRAJ_LDS=2' 'l1b:TORJ_TRAJ_LDS=1' 'l3b:TORJ_TRAJ_LDS=3' 'l1c:TORJ_TRAJ_LDS=1' 'l3c:TORJ_TRAJ_LDS=3' || exit 1
TORJ_TRAJ_LDS=3 timeout -k 10 600 python bench.py --steps 20 --no-host-api > $O/bench_l3.log 2>&1 || { tail -20 $O/bench_l3.log; exit 1; }
grep '^{' $O/bench_l3.log > $O/bench_l3.json
python -c "import json; d=json.load(open('$O/bench_l3.json')); r=d['roofline']; p=d['parity']; print('l3 bench', d['value'], r['kernel_ms'], r['frac'], p['rays_within_bar'], p['rays'], p['max_rel'])"
