#!/bin/bash
# A/B of library variants on the headline bench (kernel ms of the trace phase):
# bash scripts/gpu_ab.sh OUTDIR variant1 variant2 ... ("base" = the in-tree build)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift
mkdir -p $O
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/torj.jl_amd/build/libtorj_hip.so; else L=$PWD/torj.jl_amd/build/variants/libtorj_hip_$v.so; fi
  TORJ_HIP_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-exact --steps 3 $BENCH_ARGS > $O/$v.log 2>&1 || { echo "$v failed"; tail -5 $O/$v.log; exit 1; }
  grep '^{' $O/$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', round(d['value']/1e9,4), 'e9 ray-steps/s; trace', round(r['kernel_ms'],2), 'ms; post', round(r['deposition_kernels_ms'],2), 'ms; frac', round(r['frac'],4))"
done
