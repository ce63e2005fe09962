#!/bin/bash
# Focused GPU tests (-k expression) then optional bench configs: tools/gpu_k.sh <tag> <expr> [config...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; EXPR=$2; shift 2
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    -k "$EXPR" > $OUT/pytest.log 2>&1 || { grep -E "PASS|FAIL|Error|assert" $OUT/pytest.log | tail -30; exit 1; }
tail -2 $OUT/pytest.log
for c in "$@"; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --config $c > $OUT/bench_$c.json 2> $OUT/bench_$c.err || { tail $OUT/bench_$c.err; exit 1; }
  cat $OUT/bench_$c.json
done
