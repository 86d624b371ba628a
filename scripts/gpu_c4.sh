#!/bin/bash
# One GPU call: C4's per-shard cost (tools/c4_balance.py) and the C4 beam on one
# GPU through the bench (1 005 293 rays, strong split) -> gpurun_out/c4/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c4
mkdir -p $O
timeout -k 10 600 python -u tools/c4_balance.py > $O/c4_balance.json 2> $O/c4_balance.err || { tail -20 $O/c4_balance.err; exit 1; }
tail -3 $O/c4_balance.json
timeout -k 10 600 python -u bench.py --n-rings 291 --shard --steps 5 --warmup 1 > $O/bench_c4.log 2>&1 || { tail -20 $O/bench_c4.log; exit 1; }
grep '^{' $O/bench_c4.log | cut -c1-600
