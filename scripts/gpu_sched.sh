#!/bin/bash
# GPU tests, then one-shot vs ready-queue kernel timings over beam sizes and
# persistent-wave counts.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/sched
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
run() {  # nr sched W
  TORJ_SCHED=$2 TORJ_SCHED_W=$3 timeout -k 10 300 python bench.py --n-rings $1 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/sched/r$1_s$2_w$3.log 2>&1 || { echo fail; tail -5 gpurun_out/sched/r$1_s$2_w$3.log; exit 1; }
  python - $1 $2 $3 <<'PY'
import json,sys
nr,sch,w=sys.argv[1:]
for l in open(f"gpurun_out/sched/r{nr}_s{sch}_w{w}.log"):
    if l.startswith("{"):
        d=json.loads(l); n=d['config']['rays_per_gpu']
        print(f"rings {nr:>4} sched {sch} W {w:>5} rays {n:>7} kernel_ms {d['roofline']['kernel_ms']:8.1f} value {d['value']:.3e} frac {d['roofline']['frac']:.3f}", flush=True)
PY
}
run 92 0 0 && run 92 1 0 && run 92 1 1024 && run 92 1 1280 && run 92 1 1536 && run 92 1 2048 || exit 1
for nr in 60 130; do run $nr 0 0 && run $nr 1 0 || exit 1; done
