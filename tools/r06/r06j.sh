#!/bin/bash
# round 6 checkpoint: the whole GPU suite, then the bench lines of every config
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06j}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/gpu_benches.sh $T "c3:--config c3 --no-cpu-baseline --pmc off" \
    "c3p:--config c3 --obs packed --no-cpu-baseline --pmc off" \
    "c3ch:--config c3 --obs channels --no-cpu-baseline --pmc off" \
    "c4:--config c4 --no-cpu-baseline --pmc off" \
    "c2:--config c2 --no-cpu-baseline --pmc off" \
    "c5:--config c5 --no-cpu-baseline --pmc off" \
    "c5p:--config c5 --obs packed --no-cpu-baseline --pmc off" \
    "c5s:--config c5 --rng stream --no-cpu-baseline --pmc off" \
    "c5g:--config c5 --rng seeded --no-cpu-baseline --pmc off" || exit 1
bash tools/kt.sh $T/c3 --config c3 || exit 1
