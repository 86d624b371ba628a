#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sweep
for nr in ${RINGS:-20 60 75 92 100 110 130}; do
  timeout -k 10 300 python bench.py --n-rings $nr --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/sweep/r$nr.log 2>&1 || { echo "fail $nr"; tail -5 gpurun_out/sweep/r$nr.log; exit 1; }
  python - $nr <<'PY'
import json,sys
nr=sys.argv[1]
for l in open(f"gpurun_out/sweep/r{nr}.log"):
    if l.startswith("{"):
        d=json.loads(l); n=d['config']['rays_per_gpu']
        print(f"rings {nr:>4} rays {n:>7} waves/SIMD {n/64/1024:5.2f} kernel_ms {d['roofline']['kernel_ms']:8.1f} value {d['value']:.3e} frac {d['roofline']['frac']:.3f}")
PY
done
