#!/bin/bash
# rocprofv3 kernel-trace/stats of the default bench command, then separate PMC
# passes (never combined with tracing) of the same workload.
# usage: bash scripts/profile.sh TAG [extra bench args...]
set -o pipefail
TAG=${1:-prof}; shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
B=$GRAFT_REPO_ROOT/bench.py
run() { local name=$1; shift; local args=$1; shift; (cd /tmp && timeout -k 10 400 rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 $B $args > $OUT/$name.log 2>&1); }
run trace "--no-cpu-baseline --no-host-api --no-exact $*" --kernel-trace --stats || { echo "trace pass failed"; tail -20 $OUT/trace.log; exit 1; }
P="--steps 1 --warmup 0 --no-cpu-baseline --no-host-api --no-exact $*"
run pmc1 "$P" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU GRBM_GUI_ACTIVE || { echo pmc1 failed; tail -20 $OUT/pmc1.log; exit 1; }
run pmc2 "$P" --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA || { echo pmc2 failed; tail -20 $OUT/pmc2.log; exit 1; }
run pmc3 "$P" --pmc FETCH_SIZE || { echo pmc3 failed; tail -20 $OUT/pmc3.log; exit 1; }
run pmc4 "$P" --pmc WRITE_SIZE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT || { echo pmc4 failed; tail -20 $OUT/pmc4.log; exit 1; }
grep -h '^{' $OUT/trace.log | cut -c1-400
cat $OUT/trace/*kernel_stats.csv | head -5
