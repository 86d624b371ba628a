#!/bin/bash
# One GPU call: the driver's multi-process bench path (torchrun, one rank per
# GPU) rehearsed with 2 ranks on the one device (TORJ_BENCH_SAME_DEVICE=1: gloo
# reduce), weak and strong (C4 --shard) -> gpurun_out/trun/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/trun
mkdir -p $O
export TORJ_BENCH_SAME_DEVICE=1
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > $O/weak.log 2>&1 || { tail -30 $O/weak.log; exit 1; }
grep '^{' $O/weak.log | cut -c1-700
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --steps 3 --warmup 1 --n-rings 291 --shard > $O/strong.log 2>&1 || { tail -30 $O/strong.log; exit 1; }
grep '^{' $O/strong.log | cut -c1-700
