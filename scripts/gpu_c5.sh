#!/bin/bash
# One GPU call: the warm-model GPU tests, then the C5 bench line (with its CPU
# peer and conditioning-flagged parity) -> gpurun_out/c5/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/c5
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "warm or split" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python bench.py --absorption warm_wr --steps 5 > $O/bench_c5.log 2>&1 || { tail -20 $O/bench_c5.log; exit 1; }
grep '^{' $O/bench_c5.log | cut -c1-300
