#!/bin/bash
# Split-ring block size vs the Infinity Cache: the trace
# phase at TORJ_SPLIT_MB = 64 / 128 / 256 / 1024 (alternating), and the HBM
# bytes per launch (FETCH_SIZE, WRITE_SIZE passes, one launch each) per size
# bash scripts/gpu_ring_ab.sh OUTDIR
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
bash scripts/gpu_env_ab.sh $1/ab 'mb1024:TORJ_SPLIT_MB=1024' 'mb256:TORJ_SPLIT_MB=256' 'mb128:TORJ_SPLIT_MB=128' 'mb64:TORJ_SPLIT_MB=64' 'mb1024b:TORJ_SPLIT_MB=1024' 'mb256b:TORJ_SPLIT_MB=256' 'mb128b:TORJ_SPLIT_MB=128' 'mb64b:TORJ_SPLIT_MB=64' || exit 1
for mb in 1024 256 128 64; do
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && TORJ_SPLIT_MB=$mb timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_${mb}_$c -o p -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-api > $GRAFT_REPO_ROOT/$O/pmc_${mb}_$c.log 2>&1) || { echo "pmc $mb $c failed"; tail -5 $O/pmc_${mb}_$c.log; exit 1; }
  done
done
python tools/ring_traffic.py $O || exit 1
