#!/bin/bash
# One GPU session: parity tests, the bench line (with CPU baseline and in-run PMC
# traffic when no record of this build exists), then rocprofv3 kernel-trace / PMC
# passes over the same bench command.
# Usage: tools/gpu_round.sh <tag> [pytest -k expr]   (writes gpurun_out/<tag>/...)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-r02}
K=${2:-}
mkdir -p $R/gpurun_out/$TAG
cd $R
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${KARG[@]}" \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
timeout -k 10 900 python3 bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err \
    || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
bash tools/profile.sh $TAG/prof || exit 1
