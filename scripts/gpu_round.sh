#!/bin/bash
# One GPU call at the end of a round: the GPU suite, smoke, the 100 000-tuple
# alpha sweep, profiles of the headline (C3, split pipeline) and warm (C5) bench
# workloads, then the bench lines with their CPU baselines (C3, C5, C4 on one
# GPU) -> gpurun_out/round/ (profiles copied to profiles/$ROUND/ in the tree
# that travels back under gpurun_out/round/profiles)
cd "$GRAFT_REPO_ROOT" || exit 1
set -o pipefail
R=${ROUND:-r04}
O=gpurun_out/round
mkdir -p $O/profiles
timeout -k 10 1100 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/profiles/alpha_sweep.json 2> $O/alpha_sweep.err || { tail -20 $O/alpha_sweep.err; exit 1; }
bash scripts/profile.sh prof_c3 || exit 1
python tools/prof_summary.py gpurun_out/prof_c3 $O/profiles "k_traj|k_alpha_pts|k_tau_scan|k_split_final|k_depo_stream|k_depo_elim|k_depo_walk" || exit 1
python tools/prof_summary.py gpurun_out/prof_c3 $O/profiles k_depo_tail depo_ || exit 1
mkdir -p profiles/$R && cp $O/profiles/*.json $O/profiles/*.csv profiles/$R/ 2>/dev/null
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log | cut -c1-400
