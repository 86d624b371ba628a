#!/bin/bash
# One GPU call: profile (kernel trace + PMC passes) and bench line of the fully
# relativistic warm model (--absorption warm_fr, ~65 s per launch) ->
# gpurun_out/round_fr/, profiles copied to profiles/$ROUND/ (fr_ prefix)
cd "$GRAFT_REPO_ROOT" || exit 1
R=${ROUND:-r02}
O=gpurun_out/round_fr
mkdir -p $O/profiles
bash scripts/profile.sh prof_fr --absorption warm_fr --steps 1 --warmup 0 || exit 1
python tools/prof_summary.py gpurun_out/prof_fr $O/profiles k_trace fr_ || exit 1
mkdir -p profiles/$R && cp $O/profiles/*.json $O/profiles/*.csv profiles/$R/ 2>/dev/null
timeout -k 10 600 python bench.py --absorption warm_fr --steps 1 --warmup 0 > $O/bench_fr.log 2>&1 || { tail -20 $O/bench_fr.log; exit 1; }
grep '^{' $O/bench_fr.log | cut -c1-400
