#!/bin/bash
# PMC profile of one variant library: tools/profile_variant.sh <variant.so> <name>
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
export SAFELIFE_HIP_LIB=$R/safelife-k2_amd/build/variants/$1
NAME=$2
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 10 --warmup 2 --burnin 300 --no-cpu-baseline"
run() {
  local n=$1; shift
  timeout -k 10 300 rocprofv3 "$@" --output-format csv -d $OUT/$n -o $n -- python3 $BENCH > $OUT/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc"; return $rc
}
run kt --kernel-trace --stats || exit 1
run sq1 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
run sq2 --kernel-trace --pmc SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE || exit 1
run sq3 --kernel-trace --pmc SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_IFETCH || exit 1
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.json
