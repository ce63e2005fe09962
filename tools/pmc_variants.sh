#!/bin/bash
# Dynamic VALU / SALU / memory instruction counts per wave of every variant library in
# build/variants (one rocprofv3 --pmc pass each): tools/pmc_variants.sh <cfg> [kernel-substr]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
CFG=${1:-c5}; KS=${2:-k_env_step}
OUT=$R/gpurun_out/pmcv
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in $R/safelife-k2_amd/build/variants/*.so; do
  n=$(basename $lib .so)
  SAFELIFE_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS \
     --output-format csv -d $OUT/$n -o $n -- python3 $R/bench.py --config $CFG --steps 40 --warmup 5 --burnin 100 --no-cpu-baseline > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -5 $OUT/$n.log; exit 1; }
  python3 - $OUT/$n $KS $n <<'PY'
import csv, glob, sys
from collections import defaultdict
d, ks, name = sys.argv[1], sys.argv[2], sys.argv[3]
f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
acc = defaultdict(lambda: defaultdict(float)); n = defaultdict(int)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if ks not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in acc.items():
    w = c["SQ_WAVES"]
    print("%-10s %-40s valu/wave %8.0f salu/wave %7.0f rd/wave %6.1f wr/wave %6.1f lds/wave %6.1f" % (
        name, k.split("(")[0][-40:], c["SQ_INSTS_VALU"] / w, c["SQ_INSTS_SALU"] / w,
        c["SQ_INSTS_VMEM_RD"] / w, c["SQ_INSTS_VMEM_WR"] / w, c["SQ_INSTS_LDS"] / w))
PY
done
