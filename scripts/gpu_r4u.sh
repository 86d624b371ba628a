#!/bin/bash
# round 4: warm alpha groups of 64 lanes as the default -- the warm and split
# GPU tests, C5 at fan scale, and the C5 bench line with its parity sample
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4u
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_warm.py tests/test_gpu_split.py tests/test_gpu_c5.py -x -q --timeout 600 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 600 python bench.py --absorption warm_wr --steps 3 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log > $O/bench_c5.json
python -c "import json; d=json.load(open('$O/bench_c5.json')); r=d['roofline']; p=d['parity']; c=p['conditioning']; print('C5', d['value'], r['kernel_ms'], r['frac'], p['rays_within_bar'], p['rays'], c['rays_flagged'], c['rays_within_bar_unflagged'], c['rays_unflagged'], c['rays_out_of_bar_flagged'])"
