#!/bin/bash
# The round's second GPU call: the C5 profile and bench line, C4 on one GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
R=${ROUND:-r04}
O=gpurun_out/round
mkdir -p $O/profiles
bash scripts/profile.sh prof_c5 --absorption warm_wr || exit 1
python tools/prof_summary.py gpurun_out/prof_c5 $O/profiles "k_traj|k_alpha_warm_pts|k_tau_scan|k_split_final|k_depo_stream|k_depo_elim|k_depo_walk" c5_ || exit 1
mkdir -p profiles/$R && cp $O/profiles/c5_* profiles/$R/ 2>/dev/null
timeout -k 10 600 python bench.py --absorption warm_wr --steps 2 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log | cut -c1-300
timeout -k 10 600 python bench.py --n-rings 291 --shard --steps 3 --warmup 1 > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log | cut -c1-300
