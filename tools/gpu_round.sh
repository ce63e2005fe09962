#!/bin/bash
# One GPU session: parity tests, the bench line (with CPU baseline), then rocprofv3
# kernel-trace / PMC passes over the same bench command.
# Usage: tools/gpu_round.sh <tag>   (writes gpurun_out/<tag>/...)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r01}
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
timeout -k 10 600 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || exit 1
cat gpurun_out/$TAG/bench.json
bash tools/profile.sh $TAG/prof || exit 1
