#!/bin/bash
# Profile one bench workload on the loaded build: rocprofv3 kernel trace + the
# PMC passes (scripts/profile.sh), the per-launch summary stamped with the
# build id (tools/prof_summary.py -> profiles/$ROUND/<prefix>*), and the
# serialised pipeline's kernel times (TORJ_SPLIT_SERIAL=1).
# usage: ROUND=r05 bash scripts/gpu_prof.sh c3|c5 [extra bench args...]
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
R=${ROUND:-r05}
W=$1; shift
case $W in
  c3) PRE=""; ALPHA=k_alpha_pts; ARGS="$*" ;;
  c5) PRE="c5_"; ALPHA=k_alpha_warm_pts; ARGS="--absorption warm_wr $*" ;;
  *) echo "workload c3|c5"; exit 1 ;;
esac
O=gpurun_out/prof_$W
mkdir -p $O/profiles profiles/$R
bash scripts/profile.sh prof_$W $ARGS || exit 1
python tools/prof_summary.py gpurun_out/prof_$W $O/profiles "k_traj|$ALPHA|k_tau_scan|k_split_final|k_depo_stream|k_depo_elim|k_depo_walk" $PRE || exit 1
(cd /tmp && TORJ_SPLIT_SERIAL=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/serial -o s -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --no-exact --steps 3 $ARGS > $GRAFT_REPO_ROOT/$O/serial.log 2>&1) || { echo serial failed; tail -5 $O/serial.log; exit 1; }
f=$(find $O/serial -name '*kernel_stats.csv' | head -1); cp $f $O/profiles/${PRE}serial_kernel_stats.csv
grep -E "k_traj|k_alpha|k_tau|k_depo|k_split" $f | cut -d, -f1-4
cp $O/profiles/* profiles/$R/
