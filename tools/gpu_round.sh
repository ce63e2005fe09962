#!/bin/bash
# One GPU session: bench line (with CPU baseline) + rocprofv3 kernel trace / PMC passes.
# Usage: tools/gpu_round.sh <tag>   (writes gpurun_out/<tag>/...)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r01}
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 600 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
cat gpurun_out/$TAG/bench.json
bash tools/profile.sh $TAG/prof || exit 1
