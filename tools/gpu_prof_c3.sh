#!/bin/bash
# Full GPU test suite, then the c3 profiles (no obs, packed obs) for profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-p}
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    > gpurun_out/$TAG/pytest.log 2>&1 || { tail -40 gpurun_out/$TAG/pytest.log; exit 1; }
tail -2 gpurun_out/$TAG/pytest.log
bash tools/profile.sh ${TAG}_c3 || exit 1
bash tools/profile.sh ${TAG}_c3obs --obs packed || exit 1
