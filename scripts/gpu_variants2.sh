#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
for args in "--n-rings 60" ""; do
  echo "== $args"
  BENCH_ARGS="$args" bash scripts/run_variants.sh || exit 1
done
