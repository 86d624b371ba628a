#!/bin/bash
# GPU tests + headline bench (no CPU baseline) -> gpurun_out/quick/
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/quick
timeout -k 10 900 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/quick/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/quick/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/quick/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/quick/bench.log 2>&1 || { tail -20 gpurun_out/quick/bench.log; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/quick/bench.log"):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(f"value {d['value']:.4e} ms/step {d['ms_per_step']:.1f} kernel {r['kernel']} {r['kernel_ms']:.1f} ms frac {r['frac']:.4f} host_api {d.get('host_api',{}).get('value',0):.3e}")
PY
