#!/bin/bash
# reference-deposition parity tests, error diagnostic, and timing of both modes
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/dep
timeout -k 10 600 python -m pytest tests -x -q -m gpu -p no:cacheprovider > gpurun_out/dep/pytest.log 2>&1 || { tail -30 gpurun_out/dep/pytest.log; exit 1; }
tail -1 gpurun_out/dep/pytest.log
timeout -k 10 300 python scripts/dbg_fitdepo.py > gpurun_out/dep/err.txt 2>&1 || { cat gpurun_out/dep/err.txt; exit 1; }
cat gpurun_out/dep/err.txt
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/dep/prof -o dp -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --deposition reference --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/dep/b.log 2>&1) || { tail gpurun_out/dep/b.log; exit 1; }
head -8 $(find gpurun_out/dep/prof -name "*kernel_stats.csv") | cut -c1-150
