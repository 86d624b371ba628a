#!/bin/bash
# round 4 A/B of the trajectory / alpha / scan changes (variants), the GPU
# tests they touch, serialised kernel times, and the torchrun rehearsal
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O/profiles
timeout -k 10 900 python -u -m pytest tests/test_gpu_split.py tests/test_gpu_parity.py tests/test_gpu_c3.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/gpu_ab.sh r4e/b128 nob128 nomove noscan scan2 base nob128 nomove noscan scan2 base || exit 1
for v in base nob128; do
  if [ $v = base ]; then L=$PWD/torj.jl_amd/build/libtorj_hip.so; else L=$PWD/torj.jl_amd/build/variants/libtorj_hip_$v.so; fi
  (cd /tmp && TORJ_HIP_LIB=$L TORJ_SPLIT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/serial_$v -o s -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --steps 3 > $GRAFT_REPO_ROOT/$O/serial_$v.log 2>&1) || { echo serial $v failed; tail -5 $O/serial_$v.log; exit 1; }
  f=$(find $O/serial_$v -name '*kernel_stats.csv' | head -1); echo "serial $v"; grep -E "k_traj|k_alpha_pts|k_tau|k_depo" $f | cut -d, -f1-4
done
TORJ_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > $O/trun2.log 2>&1 || { tail -30 $O/trun2.log; exit 1; }
grep '^{' $O/trun2.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('trun2', d['value'], d['ms_per_step'], d['multi_gpu']['trace_ms_per_device'])"
