#!/bin/bash
# round 4: the Albajar node pair with hx^(2m) factored out (torj_math.hpp
# pair_term) -- its GPU tests, the 100 000-tuple sweep statistics against the
# previous build (HEAD variant), and an alternating bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_split.py tests/test_gpu_c3.py -x -v --timeout 600 --timeout-method thread -p no:cacheprovider -k "albajar or negligible or sampled_parity or split_equals or serial" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed" $O/pytest.log
timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/sweep_new.json 2> $O/sweep_new.err || { tail -5 $O/sweep_new.err; exit 1; }
TORJ_HIP_LIB=$PWD/torj.jl_amd/build/variants/libtorj_hip_head.so timeout -k 10 300 python scripts/alpha_sweep_stats.py > $O/sweep_head.json 2> $O/sweep_head.err || { tail -5 $O/sweep_head.err; exit 1; }
for f in new head; do python -c "import json; d=json.load(open('$O/sweep_$f.json')); print('$f', {k: d[k] for k in ('max_rel','p99_rel','median_rel','above_1e-10')})"; done
bash scripts/gpu_ab.sh r4c/ab head base head base || exit 1
