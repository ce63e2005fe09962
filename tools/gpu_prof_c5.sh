#!/bin/bash
# 128x128 parity tests, then the c5 profile (kernel trace + PMC passes) for profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-p5}
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    -k "128 or tiny_batches" > gpurun_out/$TAG/pytest.log 2>&1 || { tail -30 gpurun_out/$TAG/pytest.log; exit 1; }
tail -1 gpurun_out/$TAG/pytest.log
bash tools/profile.sh ${TAG}_c5 --config c5 || exit 1
