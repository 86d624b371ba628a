#!/bin/bash
# round 4: pinned, pipelined torj_trace_beam staging + per-replica timing, the
# GL node records; GPU tests, the full default bench line, and the N = 2 lines
# of both launch paths rehearsed on the one device
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests/test_gpu_beam.py tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_c3.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -2
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
grep '^{' $O/bench.log > $O/bench.json
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['kernel_ms'], d['roofline']['frac']); print('library_path', d['library_path']); print('host_api', d['host_api']); print('beam_c4', d.get('host_api_beam_c4')); print('parity', {k: d['parity'][k] for k in ('rays','rays_within_bar','max_rel')})"
TORJ_BEAM_SAME_DEVICE=1 timeout -k 10 600 python bench.py --gpus 2 --steps 5 --warmup 1 > $O/lib2.log 2>&1 || { tail -20 $O/lib2.log; exit 1; }
grep '^{' $O/lib2.log > $O/lib2.json
python -c "import json; d=json.load(open('$O/lib2.json')); print('lib2', d['value'], d['multi_gpu'], d['parity']['rays_within_bar'], d['parity']['rays'])"
TORJ_BENCH_SAME_DEVICE=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 > $O/trun2.log 2>&1 || { tail -30 $O/trun2.log; exit 1; }
grep '^{' $O/trun2.log > $O/trun2.json
python -c "import json; d=json.load(open('$O/trun2.json')); print('trun2', d['value'], d['multi_gpu'], d['parity']['rays_within_bar'], d['parity']['rays'])"
