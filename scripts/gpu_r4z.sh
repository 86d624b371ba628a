#!/bin/bash
# round 4, final call on HEAD: the GPU suite, smoke, the round profile (C3),
# the serialised kernel times, and the bench lines of C3, C5 and C4 (one GPU)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4z
mkdir -p $O/profiles
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/profiles/alpha_sweep.json 2> $O/alpha_sweep.err || { tail -5 $O/alpha_sweep.err; exit 1; }
bash scripts/profile.sh prof_r4z || exit 1
python tools/prof_summary.py gpurun_out/prof_r4z $O/profiles "k_traj|k_alpha_pts|k_tau_scan|k_split_final|k_depo_stream|k_depo_elim|k_depo_walk" || exit 1
python tools/prof_summary.py gpurun_out/prof_r4z $O/profiles k_depo_tail depo_ || exit 1
(cd /tmp && TORJ_SPLIT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/serial -o s -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --steps 3 > $GRAFT_REPO_ROOT/$O/serial.log 2>&1) || { echo serial failed; tail -5 $O/serial.log; exit 1; }
f=$(find $O/serial -name '*kernel_stats.csv' | head -1); cp $f $O/profiles/serial_kernel_stats.csv; grep -E "k_traj|k_alpha_pts|k_tau|k_depo" $f | cut -d, -f1-4
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log > $O/bench_c3.json
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; p=d['parity']; print('C3', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], p['rays_within_bar'], p['rays']); print('beam_c4', d.get('host_api_beam_c4', {}).get('value'))"
timeout -k 10 600 python bench.py --absorption warm_wr --steps 3 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log > $O/bench_c5.json
python -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; p=d['parity']; print('C5', d['value'], r['kernel_ms'], r['frac'], p.get('rays_within_bar'), p.get('rays'), p.get('conditioning', {}).get('rays_within_bar_unflagged'))"
timeout -k 10 600 python bench.py --n-rings 291 --shard --steps 3 --warmup 1 --no-host-api > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log > $O/bench_c4_1gpu.json
python -c "import json; d=json.load(open('$O/bench_c4_1gpu.json')); r=d['roofline']; print('C4', d['value'], d['ms_per_step'], r['kernel_ms'], d['parity']['rays_within_bar'], d['parity']['rays'])"
