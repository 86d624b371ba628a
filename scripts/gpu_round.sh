#!/bin/bash
# One GPU call: GPU tests, profiles of the headline (C3) and warm (C5) bench
# workloads, then both bench lines with their CPU baselines -> gpurun_out/round/
# (copy gpurun_out/round/profiles/* to profiles/<round>/ afterwards)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/round
mkdir -p $O/profiles
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
bash scripts/profile.sh prof_c3 || exit 1
python tools/prof_summary.py gpurun_out/prof_c3 $O/profiles k_trace || exit 1
python tools/prof_summary.py gpurun_out/prof_c3 $O/profiles k_fit_depo depo_ || exit 1
bash scripts/profile.sh prof_c5 --absorption warm_wr || exit 1
python tools/prof_summary.py gpurun_out/prof_c5 $O/profiles k_trace c5_ || exit 1
cp $O/profiles/*.json $O/profiles/*.csv profiles/${ROUND:-r01}/ 2>/dev/null
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log
timeout -k 10 600 python bench.py --absorption warm_wr --steps 2 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log
timeout -k 10 600 python bench.py --absorption warm_fr --steps 1 --no-cpu-baseline > $O/bench_warm_fr.log 2>&1 || { tail -20 $O/bench_warm_fr.log; exit 1; }
grep '^{' $O/bench_warm_fr.log
