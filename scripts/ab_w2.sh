#!/bin/bash
# A/B of warm alpha-kernel variants on the C5 bench (split path forced):
# bash scripts/ab_w2.sh base w3 ...  (variants from scripts/mkvariant.py); ABS env: warm_wr (default)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/w2
ab=${ABS:-warm_wr}
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/torj.jl_amd/build/libtorj_hip.so; else L=$PWD/torj.jl_amd/build/variants/libtorj_hip_$v.so; fi
  TORJ_SPLIT_WARM=1 TORJ_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-api --steps 2 --warmup 1 --absorption $ab > gpurun_out/w2/${v}_${ab}.log 2>&1 || { echo "$v $ab failed"; tail -3 gpurun_out/w2/${v}_${ab}.log; exit 1; }
  grep '^{' gpurun_out/w2/${v}_${ab}.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v $ab', round(d['roofline']['kernel_ms'],2), 'ms', round(d['value']/1e9,4), 'e9')"
done
