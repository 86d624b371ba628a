#!/bin/bash
# round 4: cell records per metre (no 1/h per gradient field), rsqrt-based
# reciprocal square roots in the RHS and the Albajar prologue, the exact-zero
# test without a square root -- the GPU suite, the 100 000-tuple alpha sweep,
# an alternating A/B against HEAD and the profile of the new default
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4p
mkdir -p $O/profiles
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/alpha_sweep.json 2> $O/alpha_sweep.err || { tail -5 $O/alpha_sweep.err; exit 1; }
python -c "import json; d=json.load(open('$O/alpha_sweep.json')); print({k: d[k] for k in ('max_rel','p99_rel','median_rel','above_1e-10')})"
bash scripts/gpu_ab.sh r4p/ab head base head base head base || exit 1
bash scripts/profile.sh prof_r4p || exit 1
python tools/prof_summary.py gpurun_out/prof_r4p $O/profiles "k_traj|k_alpha_pts|k_tau_scan|k_split_final|k_depo_stream|k_depo_elim|k_depo_walk" || exit 1
python tools/prof_summary.py gpurun_out/prof_r4p $O/profiles k_depo_tail depo_ || exit 1
