set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/t2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o tr -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --steps 3 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1) || { tail -5 $O/trace.log; exit 1; }
f=$(find $O/trace -name '*kernel_trace.csv' | head -1); python tools/timeline.py $f 3
(cd /tmp && TORJ_SPLIT_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/serial -o s -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-host-api --steps 3 > $GRAFT_REPO_ROOT/$O/serial.log 2>&1) || { tail -5 $O/serial.log; exit 1; }
f=$(find $O/serial -name '*kernel_stats.csv' | head -1); grep -E "k_traj|k_alpha|k_tau|k_depo|k_split" $f | cut -d, -f1-4
