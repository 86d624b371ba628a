#!/bin/bash
# A/B of runtime switches on the headline bench (kernel ms of the trace phase):
# bash scripts/gpu_env_ab.sh OUTDIR 'name:VAR=1 VAR2=2' 'base:' ...
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/$1; shift
mkdir -p $O
for spec in "$@"; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-host-api --no-exact --steps 3 $BENCH_ARGS > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', round(d['value']/1e9,4), 'e9 ray-steps/s; trace', round(r['kernel_ms'],2), 'ms; post', round(r['deposition_kernels_ms'],2), 'ms; frac', round(r['frac'],4))"
done
