#!/bin/bash
# The two N = 2 rehearsals on one MI355X (-> gpurun_out/reh/): torchrun with two
# ranks on the one device (TORJ_BENCH_SAME_DEVICE=1, gloo reduce) and the library
# path with two replicas on device 0 (TORJ_BEAM_SAME_DEVICE=1)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/reh
mkdir -p $O
TORJ_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > $O/torchrun2.log 2>&1 || { tail -30 $O/torchrun2.log; exit 1; }
grep '^{' $O/torchrun2.log > $O/bench_torchrun2_same_device_rehearsal.json
TORJ_BEAM_SAME_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 1 > $O/lib2.log 2>&1 || { tail -30 $O/lib2.log; exit 1; }
grep '^{' $O/lib2.log > $O/bench_lib2_same_device_rehearsal.json
python -c "
import json
for f in ('torchrun2', 'lib2'):
    d = json.load(open('$O/bench_' + f + '_same_device_rehearsal.json'))
    print(f, d['value'], d['config'].get('build_id'), {k: d['multi_gpu'].get(k) for k in ('device', 'rccl_nranks', 'rccl_rank', 'pg_rank', 'pg_size', 'backend')})
"
