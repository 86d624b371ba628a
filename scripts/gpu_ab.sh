#!/bin/bash
# A/B of library variants on one bench command: bash scripts/gpu_ab.sh "<bench args>" name...
# (name "main" = torj.jl_amd/build/libtorj_hip.so, else build/variants/libtorj_hip_<name>.so)
cd "$GRAFT_REPO_ROOT" || exit 1
ARGS=$1; shift
mkdir -p gpurun_out/ab
for v in "$@"; do
  if [ "$v" = main ]; then L=torj.jl_amd/build/libtorj_hip.so; else L=torj.jl_amd/build/variants/libtorj_hip_$v.so; fi
  TORJ_HIP_LIB=$PWD/$L timeout -k 10 400 python bench.py --no-cpu-baseline $ARGS > gpurun_out/ab/$v.log 2>&1 || { tail -20 gpurun_out/ab/$v.log; exit 1; }
  echo -n "$v: "; python tools/bench_brief.py gpurun_out/ab/$v.log
done
