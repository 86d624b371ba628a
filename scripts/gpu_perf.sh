#!/bin/bash
# One GPU call: a GPU test subset, the headline bench line, its rocprof trace +
# PMC profile (-> profiles/$ROUND/), an A/B of the negligible-harmonic skip
# (TORJ_NEGL_SKIP=0 / 1, alternating) and the serialised pipeline's kernel times.
cd "$GRAFT_REPO_ROOT" || exit 1
R=${ROUND:-r04}
O=gpurun_out/perf
mkdir -p $O/profiles
K=${PYTEST_K:-"negligible or split or c3 or deposition"}
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu -k "$K" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 400 python bench.py > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log | cut -c1-400
for i in 1 2; do
  for s in 0 1; do
    TORJ_NEGL_SKIP=$s timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-api --steps 5 > $O/ab_skip$s.$i.log 2>&1 || { tail -5 $O/ab_skip$s.$i.log; exit 1; }
    grep '^{' $O/ab_skip$s.$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('skip=$s', round(d['value']/1e9,4), 'e9; trace', round(r['kernel_ms'],2), 'ms; frac', round(r['frac'],4), 'ref-alg TF', round(d['work_equivalent']['reference_algorithm_equivalent_TFLOPs'],2))"
  done
done
bash scripts/profile.sh prof_c3 || exit 1
python tools/prof_summary.py gpurun_out/prof_c3 $O/profiles "k_traj|k_alpha_pts|k_tau_scan|k_split_final|k_depo_stream" || exit 1
python tools/prof_summary.py gpurun_out/prof_c3 $O/profiles k_depo_tail depo_ || exit 1
(cd /tmp && TORJ_SPLIT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_serial -o serial -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --steps 3 > $GRAFT_REPO_ROOT/$O/serial.log 2>&1) || { echo serial failed; tail -5 $O/serial.log; exit 1; }
cp gpurun_out/prof_serial/*kernel_stats.csv $O/profiles/serial_kernel_stats.csv 2>/dev/null
head -8 $O/profiles/serial_kernel_stats.csv
mkdir -p profiles/$R && cp $O/profiles/*.json $O/profiles/*.csv profiles/$R/ 2>/dev/null
echo done
