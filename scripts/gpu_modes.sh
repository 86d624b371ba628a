#!/bin/bash
# headline bench in each integrator / deposition mode
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/modes
for m in "rk4 reference" "rk4 binned" "adaptive reference"; do
  set -- $m
  timeout -k 10 400 python bench.py --no-cpu-baseline --integrator $1 --deposition $2 > gpurun_out/modes/$1_$2.log 2>&1 || { tail gpurun_out/modes/$1_$2.log; exit 1; }
  python - $1 $2 <<'PY'
import json, sys
for l in open(f"gpurun_out/modes/{sys.argv[1]}_{sys.argv[2]}.log"):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(sys.argv[1:], f"value {d['value']:.4e} ms/step {d['ms_per_step']:.1f} trace {r['kernel_ms']:.1f} depo {r['deposition_kernels_ms']:.1f} frac {r['frac']:.3f} rhs/step {d['work_counters']['rhs_evals']/d['work_counters']['ray_steps']:.2f}")
PY
done
