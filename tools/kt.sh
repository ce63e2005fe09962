#!/bin/bash
# Kernel-trace stats of one bench command (run on the GPU box):
#   tools/kt.sh <out_name> [bench args...]  -> gpurun_out/<out_name>/kt/*kernel_stats.csv
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
NAME=$1; shift
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- \
    python3 $R/bench.py --steps 100 --warmup 10 --no-cpu-baseline --pmc off "$@" > $OUT/kt.log 2>&1
rc=$?
find $OUT/kt -name "*kernel_trace.csv" -delete
f=$(find $OUT/kt -name "*kernel_stats.csv" | head -1)
[ -n "$f" ] && python3 -c "
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print('%-60s n=%6s avg=%9.1f us tot=%8.1f ms' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
" $f
exit $rc
