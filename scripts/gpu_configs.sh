#!/bin/bash
# bench lines of the side configurations (no CPU baseline) -> gpurun_out/configs/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/configs
mkdir -p $O
i=0
for args in "--deposition binned" "--n-rings 14 --min-az 5" "--mode -1" "--integrator adaptive"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 $args > $O/$i.log 2>&1 || { echo "[$args] failed"; tail -20 $O/$i.log; exit 1; }
  echo -n "[$args] "; python tools/bench_brief.py $O/$i.log
done
