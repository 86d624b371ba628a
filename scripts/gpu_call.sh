#!/bin/bash
# One development call on the GPU box (round 6): optional GPU tests (PYTEST_K,
# PYTEST_FILES), an alternating env / library A/B (AB specs 'name:VAR=1 ...',
# TORJ_HIP_LIB selects a variant library), and optionally the default bench
# line (FULL_BENCH=1).  Stops at the first step that did not end normally (a
# pytest failure, rc 1, is reported and the call goes on).
# usage: OUT=name [PYTEST_K=...] [AB="spec1 | spec2 | ..."] [REPS=2] [FULL_BENCH=1] bash scripts/gpu_call.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-call}
mkdir -p $O
if [ -n "$PYTEST_K" ] || [ -n "$PYTEST_FILES" ]; then
  timeout -k 10 ${PYTEST_T:-700} python -u -m pytest ${PYTEST_FILES:-tests} -x -v ${PYTEST_S:+-s} -m gpu ${PYTEST_K:+-k "$PYTEST_K"} \
      --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
  rc=$?
  tail -4 $O/pytest.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stop"; exit $rc; fi
  [ $rc -eq 1 ] && grep -E "^(FAILED|ERROR)|Error|assert" $O/pytest.log | head -20
fi
if [ -n "$AB" ]; then
  IFS='|' read -ra SPECS <<< "$AB"
  for rep in $(seq 1 ${REPS:-2}); do
    for spec in "${SPECS[@]}"; do
      spec=$(echo $spec | xargs)
      name=${spec%%:*}; envs=${spec#*:}
      env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-api --no-exact --steps ${AB_STEPS:-3} $BENCH_ARGS > $O/${name}_$rep.log 2>&1 || { echo "$name failed"; tail -5 $O/${name}_$rep.log; exit 1; }
      grep '^{' $O/${name}_$rep.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', round(d['value']/1e9,4), 'e9 ray-steps/s; trace', round(r['kernel_ms'],2), 'ms; post', round(r['deposition_kernels_ms'],2), 'ms; step', round(d['ms_per_step'],2), 'frac', round(r['frac'],4))" | tee -a $O/ab.txt
    done
  done
fi
if [ -n "$FULL_BENCH" ]; then
  timeout -k 10 600 python bench.py $FULL_ARGS > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
  grep '^{' $O/bench.log > $O/bench.json
  python - <<'PY'
import json, os
d = json.load(open(os.environ.get("O_JSON", "gpurun_out/" + os.environ.get("OUT", "call") + "/bench.json")))
r, p = d["roofline"], d.get("parity", {})
print("bench", d["value"], d["ms_per_step"], r["kernel_ms"], r["deposition_kernels_ms"], r["frac"])
print("parity", {k: p.get(k) for k in ("rays", "rays_within_bar", "max_rel_tau", "max_rel_tau_unfloored", "max_rel_tau_resolvable", "rays_tau_resolvable")})
e = d.get("exact")
if e:
    print("exact", {k: e.get(k) for k in ("value", "trace_ms", "deposition_ms", "headline_over_exact", "status_equal_headline", "xN_equal_headline", "max_abs_tau_diff_headline")})
    ep = e.get("parity", {})
    print("exact parity", {k: ep.get(k) for k in ("rays_within_bar", "max_rel_tau", "max_rel_tau_unfloored", "max_rel_tau_resolvable")})
PY
fi
