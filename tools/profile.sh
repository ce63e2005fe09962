#!/bin/bash
# Kernel trace + PMC passes over the headline bench command (run on the GPU box).
# Usage: tools/profile.sh <out_dir_name> [extra bench args...]
# Writes gpurun_out/<name>/{kt,fetch,write,sq1,sq2,tcc}/ and summary.json, whose
# "last_k" fields average the bench's timed window (its last --steps launches).
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=${1:-prof}; shift || true
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
STEPS=200
BENCH="$R/bench.py --steps $STEPS --warmup 20 --no-cpu-baseline --pmc off $*"
run() {  # name, rocprof args...
  local n=$1; shift
  timeout -k 10 400 rocprofv3 "$@" --output-format csv -d $OUT/$n -o $n -- python3 $BENCH > $OUT/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; return $rc
}
run kt --kernel-trace --stats || exit 1
run fetch --kernel-trace --pmc FETCH_SIZE || exit 1
run write --kernel-trace --pmc WRITE_SIZE || exit 1
run sq1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
run sq2 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE || exit 1
python3 $R/tools/pmc_summary.py $OUT --last $STEPS > $OUT/summary.json
# the per-launch traces are large (gpurun copies back at most 64 MiB): keep the
# kernel-trace pass's stats and the summary, drop the PMC passes' raw CSVs
for n in fetch write sq1 sq2; do find $OUT/$n -name "*counter_collection.csv" -delete; find $OUT/$n -name "*kernel_trace.csv" -delete; done
find $OUT/kt -name "*kernel_trace.csv" -size +8M -exec gzip {} \;
