#!/bin/bash
# A/B timing of variant libraries on the GPU box: tools/ab_run.sh <tag> "<bench args>" name...
# Each variant runs bench.py once under its own time limit; the first failure ends the run.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; ARGS=$2; shift 2
mkdir -p $R/gpurun_out/$TAG
cd $R
for v in "$@"; do
  SAFELIFE_HIP_LIB=$R/variants/$v.so timeout -k 10 300 python3 bench.py $ARGS --no-cpu-baseline --pmc off \
      > gpurun_out/$TAG/$v.json 2> gpurun_out/$TAG/$v.err || { echo "$v failed"; tail -5 gpurun_out/$TAG/$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', d['roofline'].get('kernel_ms'))" gpurun_out/$TAG/$v.json $v
done
