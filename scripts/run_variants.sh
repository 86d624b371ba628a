#!/bin/bash
# time every built variant with the headline bench (no CPU baseline)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/variants
for so in torj.jl_amd/build/variants/libtorj_hip_*.so; do
  name=$(basename $so .so); name=${name#libtorj_hip_}
  TORJ_HIP_LIB=$PWD/$so timeout -k 10 240 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $BENCH_ARGS > gpurun_out/variants/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/variants/$name.log; exit 1; }
  python - "$name" <<'PY'
import json,sys
name=sys.argv[1]
for l in open(f"gpurun_out/variants/{name}.log"):
    if l.startswith("{"):
        d=json.loads(l); print(f"{name:10s} value {d['value']:.4e} kernel_ms {d['roofline']['kernel_ms']:.1f} frac {d['roofline']['frac']:.3f}")
PY
done
