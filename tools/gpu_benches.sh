#!/bin/bash
# Bench lines on the GPU box: tools/gpu_benches.sh <tag> "<name>:<bench args>" ...
# Each line runs under its own time limit into gpurun_out/<tag>/bench_<name>.json; the
# first failure ends the run.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
cd $R
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 600 python3 bench.py $args > gpurun_out/$TAG/bench_$name.json 2> gpurun_out/$TAG/bench_$name.err \
      || { echo "$name failed"; tail -5 gpurun_out/$TAG/bench_$name.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], round(d['value']/1e6,4), 'M env-steps/s', d['ms_per_step'], 'ms/step', r.get('kernel'), r.get('kernel_ms'), 'ms frac', r['frac'], 'traffic', r['traffic'])" gpurun_out/$TAG/bench_$name.json $name
done
