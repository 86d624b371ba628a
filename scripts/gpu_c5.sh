#!/bin/bash
# warm GPU tests + the C5 bench line (no CPU baseline) -> gpurun_out/c5/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 600 python -m pytest tests/test_gpu_warm.py tests/test_gpu_parity.py -x -q -m gpu -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python bench.py --no-cpu-baseline --absorption warm_wr --steps 2 "$@" > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
python - $O/bench_c5.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); r = d["roofline"]
        print(f"value {d['value']:.4e} kernel {r['kernel']} {r['kernel_ms']:.1f} ms")
PY
