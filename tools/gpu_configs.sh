#!/bin/bash
# Bench every BASELINE config on one GPU (no CPU baseline except c3):
# tools/gpu_configs.sh <tag> [configs...]   -> gpurun_out/<tag>/bench_<cfg>.json
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-cfg}; shift || true
CFGS=${*:-c3 c2 c4 c5}
mkdir -p $R/gpurun_out/$TAG
cd $R
for c in $CFGS; do
  extra="--no-cpu-baseline"
  [ "$c" = c3 ] && extra=""
  timeout -k 10 300 python3 bench.py --config $c $extra > gpurun_out/$TAG/bench_$c.json \
      2> gpurun_out/$TAG/bench_$c.err || { tail -20 gpurun_out/$TAG/bench_$c.err; exit 1; }
  cat gpurun_out/$TAG/bench_$c.json
done
