#!/bin/bash
# Wave-cycle attribution of a bench command's step kernel (run on the GPU box):
#   tools/profile_sq.sh <out_name> [bench args...]
# Passes (each its own rocprofv3 run, at most 8 SQ counters, KILL-bounded):
#   a  the disjoint split WAVE_CYCLES = WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
#      (MI355X_MICROARCH.md: parked on s_waitcnt / issue-stalled / issuing), plus the
#      LDS issue-stall sub-bucket and the instruction counts;
#   b  what is issuing: ACTIVE_INST_{VALU,SCA,LDS,VMEM,FLAT,EXP,MISC}, LDS bank conflicts;
#   c  instruction mix: SALU, SMEM, LDS, VMEM read / write, branch, and GRBM_GUI_ACTIVE.
# Writes gpurun_out/<name>/<pass>/ and summary.json (tools/pmc_summary.py).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=$1; shift
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
STEPS=100
BENCH="$R/bench.py --steps $STEPS --warmup 10 --no-cpu-baseline --pmc off $*"
run() {  # name, counters...
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d $OUT/$n -o $n -- python3 $BENCH > $OUT/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; return $rc
}
run sqa SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU || exit 1
run sqb SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_MISC SQ_LDS_BANK_CONFLICT SQ_WAVES || exit 1
run sqc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE || exit 1
python3 $R/tools/pmc_summary.py $OUT --last $STEPS > $OUT/summary.json
for n in sqa sqb sqc; do find $OUT/$n -name "*counter_collection.csv" -delete; find $OUT/$n -name "*kernel_trace.csv" -delete; done
