#!/bin/bash
# round 4: 1/Y from 1/|B| in the refractive-index partials (in-tree build) --
# the GPU suite and the alpha sweep (with the cell tile copy by record); the degree-8 node exponential (variant e8) -- its alpha tests
# and the 100 000-tuple sweep; alternating A/B head / base / e8
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4q
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/sweep_base.json 2> $O/sweep_base.err || { tail -5 $O/sweep_base.err; exit 1; }
python -c "import json; d=json.load(open('$O/sweep_base.json')); print('base sweep', {k: d[k] for k in ('max_rel','p99_rel','median_rel','above_1e-10')})"
E8=$PWD/torj.jl_amd/build/variants/libtorj_hip_e8.so
TORJ_HIP_LIB=$E8 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c3.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "albajar or sampled_parity" > $O/pytest_e8.log 2>&1 || { tail -30 $O/pytest_e8.log; exit 1; }
tail -1 $O/pytest_e8.log
TORJ_HIP_LIB=$E8 timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/sweep_e8.json 2> $O/sweep_e8.err || { tail -5 $O/sweep_e8.err; exit 1; }
python -c "import json; d=json.load(open('$O/sweep_e8.json')); print('e8 sweep', {k: d[k] for k in ('max_rel','p99_rel','median_rel','above_1e-10')})"
bash scripts/gpu_ab.sh r4q/ab head base e8 head base e8 head base e8 || exit 1
