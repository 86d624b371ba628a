#!/bin/bash
# GPU tests, then the headline bench and the warm-absorption (C5) bench lines
# (no CPU baseline) -> gpurun_out/warm/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/warm
mkdir -p $O
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
show() {
python - "$1" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(f"{d['config']['workload'][:60]}: value {d['value']:.4e} ms/step {d['ms_per_step']:.1f} "
              f"kernel {r['kernel']} {r['kernel_ms']:.1f} ms frac {r['frac']} status {d['config']['ray_status_counts']}")
PY
}
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c3.log 2>&1 || { tail -20 $O/bench_c3.log; exit 1; }
show $O/bench_c3.log
timeout -k 10 400 python bench.py --no-cpu-baseline --absorption warm_wr --steps 2 "$@" > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
show $O/bench_c5.log
timeout -k 10 400 python bench.py --no-cpu-baseline --absorption warm_fr --steps 1 --warmup 0 "$@" > $O/bench_warm_fr.log 2>&1 || { tail -20 $O/bench_warm_fr.log; exit 1; }
show $O/bench_warm_fr.log
