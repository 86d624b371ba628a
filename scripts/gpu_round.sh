#!/bin/bash
# The round's measurement on one MI355X, in two gpurun calls (each within the
# call limit):  bash scripts/gpu_round.sh A   the GPU suite, smoke, the
# 100 000-tuple alpha sweep, the C3 profile (scripts/gpu_prof.sh: trace, PMC
# passes, serialised kernels, build-id stamped summaries) and the C3 bench line;
#               bash scripts/gpu_round.sh B   the C5 profile and bench line, C4
# on one GPU.  Everything under gpurun_out/round/ (copy the profiles and lines
# into profiles/$ROUND/).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=${ROUND:-r05}
O=gpurun_out/round
mkdir -p $O
case ${1:-A} in
A)
  timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
  timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/alpha_sweep.json 2> $O/alpha_sweep.err || { tail -20 $O/alpha_sweep.err; exit 1; }
  ROUND=$R timeout -k 10 900 bash scripts/gpu_prof.sh c3 || exit 1
  timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
  grep '^{' $O/bench_c3.log > $O/bench_c3.json
  python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; p=d['parity']; print('C3', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['traffic_source'], p['rays_within_bar'], p['rays'])"
  ;;
B)
  ROUND=$R timeout -k 10 900 bash scripts/gpu_prof.sh c5 || exit 1
  timeout -k 10 600 python bench.py --absorption warm_wr --steps 3 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
  grep '^{' $O/bench_c5.log > $O/bench_c5.json
  python -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; p=d['parity']; c=p.get('conditioning', {}); print('C5', d['value'], r['kernel_ms'], r['frac'], r['traffic_source'], c.get('rays_within_bar_all'), p.get('rays'), c.get('rays_within_bar_unflagged'), c.get('rays_unflagged'))"
  timeout -k 10 600 python bench.py --n-rings 291 --shard --steps 3 --warmup 1 > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
  grep '^{' $O/bench_c4.log > $O/bench_c4_1gpu.json
  python -c "import json; d=json.load(open('$O/bench_c4_1gpu.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r['kernel_ms'], d['parity']['rays_within_bar'], d['parity']['rays'])"
  ;;
esac
