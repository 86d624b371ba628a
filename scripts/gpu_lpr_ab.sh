#!/bin/bash
# small-beam A/B: 16 lanes per ray (automatic) vs one lane per ray (TORJ_LPR=1) -> gpurun_out/lpr/
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/lpr
mkdir -p $O
for a in "--n-rings 14 --min-az 5" "--n-rings 30 --min-az 7" "--n-rings 14 --min-az 5 --absorption none"; do
  for lpr in 0 1; do
    f=$O/$(echo "$a $lpr" | tr -c 'a-z0-9' _).log
    TORJ_LPR=$lpr timeout -k 10 200 python bench.py --no-cpu-baseline --steps 5 $a > $f 2>&1 || { tail -20 $f; exit 1; }
    echo -n "[$a] TORJ_LPR=$lpr "; python tools/bench_brief.py $f
  done
done
