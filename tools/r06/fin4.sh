#!/bin/bash
# round 6 final, part 4: the per-config bench lines
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06fin}
cd $R
bash tools/gpu_benches.sh $T "c1:--config c1 --no-cpu-baseline --pmc off" \
    "c2:--config c2 --no-cpu-baseline --pmc off" \
    "c3:--config c3 --no-cpu-baseline --pmc off" \
    "c3p:--config c3 --obs packed --no-cpu-baseline --pmc off" \
    "c3ch:--config c3 --obs channels --no-cpu-baseline --pmc off" \
    "c4:--config c4 --no-cpu-baseline --pmc off" \
    "c5:--config c5 --no-cpu-baseline --pmc off" \
    "c5p:--config c5 --obs packed --no-cpu-baseline --pmc off" \
    "c5s:--config c5 --rng stream --no-cpu-baseline --pmc off" \
    "c5g:--config c5 --rng seeded --no-cpu-baseline --pmc off"
