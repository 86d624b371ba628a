#!/bin/bash
# round 4: psi of each step's end from the next step's stage-0 stencil (k_traj)
# -- the GPU suite and smoke on it, an alternating A/B against the previous
# build (variant "head"), then the round profile and the full bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4h
mkdir -p $O/profiles
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash scripts/gpu_ab.sh r4h/ab head base head base head base || exit 1
bash scripts/profile.sh prof_r4h || exit 1
python tools/prof_summary.py gpurun_out/prof_r4h $O/profiles "k_traj|k_alpha_pts|k_tau_scan|k_split_final|k_depo_stream|k_depo_elim|k_depo_walk" || exit 1
python tools/prof_summary.py gpurun_out/prof_r4h $O/profiles k_depo_tail depo_ || exit 1
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log > $O/bench_c3.json
python -c "import json; d=json.load(open('$O/bench_c3.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], d['parity']['rays_within_bar'], d['parity']['rays'])"
