#!/bin/bash
# A/B of environment settings on one bench command:
#   bash scripts/gpu_env_ab.sh "<bench args>" "ENV=VAL ..." "ENV=VAL ..." ...  ("-" = none)
cd "$GRAFT_REPO_ROOT" || exit 1
ARGS=$1; shift
mkdir -p gpurun_out/envab
i=0
for e in "$@"; do
  i=$((i+1))
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 400 python bench.py --no-cpu-baseline $ARGS > gpurun_out/envab/$i.log 2>&1 || { tail -20 gpurun_out/envab/$i.log; exit 1; }
  echo -n "[$e] "; python tools/bench_brief.py gpurun_out/envab/$i.log
done
