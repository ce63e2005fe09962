#!/bin/bash
# round 6, first GPU pass: the plane-mode tests (stale-board fixes, fused 128x128 views),
# then the C5 lines with and without packed views and their kernel stats
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=r06a
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
    -k "board_planes or feed or golden128 or reference_without_obs or g7" \
    > gpurun_out/$T/pytest.log 2>&1 || { tail -60 gpurun_out/$T/pytest.log; exit 1; }
tail -3 gpurun_out/$T/pytest.log
bash tools/gpu_benches.sh $T "c5:--config c5 --no-cpu-baseline --pmc off" \
    "c5p:--config c5 --obs packed --no-cpu-baseline --pmc off" || exit 1
bash tools/kt.sh $T/c5p --config c5 --obs packed || exit 1
