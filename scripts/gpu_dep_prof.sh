#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/depprof
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/depprof -o dp -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --deposition reference --steps 2 > $GRAFT_REPO_ROOT/gpurun_out/depprof/b.log 2>&1) || { tail gpurun_out/depprof/b.log; exit 1; }
head -8 $(find gpurun_out/depprof -name "*kernel_stats.csv")
