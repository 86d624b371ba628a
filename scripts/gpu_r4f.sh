#!/bin/bash
# C4 (1 005 293 rays) on one MI355X, device-resident: one launch (default) vs
# ray batches of ~130k rays (TORJ_WS_GB=15) vs a 4 GiB split-ring slot budget
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4f
mkdir -p $O
for spec in 'one:' 'sb131:TORJ_SPLIT_BATCH=131072' 'ws15:TORJ_WS_GB=15' 'mb4096:TORJ_SPLIT_MB=4096' 'one2:' 'sb131b:TORJ_SPLIT_BATCH=131072' 'sb262:TORJ_SPLIT_BATCH=262144'; do
  name=${spec%%:*}; envs=${spec#*:}
  env $envs timeout -k 10 300 python bench.py --n-rings 291 --shard --steps 3 --warmup 1 --no-cpu-baseline --no-host-api > $O/$name.log 2>&1 || { echo "$name failed"; tail -5 $O/$name.log; exit 1; }
  grep '^{' $O/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$name', round(d['value']/1e9,4), 'e9; ms', round(d['ms_per_step'],1), 'trace', round(r['kernel_ms'],1), 'post', round(r['deposition_kernels_ms'],1))"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_split.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "streamed" > $O/pytest_stream.log 2>&1 || { tail -30 $O/pytest_stream.log; exit 1; }
tail -1 $O/pytest_stream.log
bash scripts/gpu_env_ab.sh r4f/depo3 's1:TORJ_DEPO_STREAM=1' 's3:TORJ_DEPO_STREAM=3' 's1b:TORJ_DEPO_STREAM=1' 's3b:TORJ_DEPO_STREAM=3' || exit 1
