#!/bin/bash
# round 4: the full GPU suite, smoke and the default bench line with the
# cell-tiled trajectory kernel as the default (TORJ_TRAJ_LDS=3)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log > $O/bench_c3.json
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; p=d['parity']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], p['rays_within_bar'], p['rays'], p['max_rel']); print('library_path', d.get('library_path')); print('beam_c4', d.get('host_api_beam_c4'))"
