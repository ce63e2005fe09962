#!/bin/bash
# GPU parity tests (one process, per-test timeout) then the per-config benches.
# tools/gpu_session.sh <tag> [configs...]
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-s}; shift || true
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -3 gpurun_out/$TAG/pytest.log
bash tools/gpu_configs.sh $TAG "$@"
