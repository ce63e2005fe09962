#!/bin/bash
# round 6 final, part 3: profiles of C5 (Philox, packed views, replay, seeded) and C2
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06fin}
cd $R
bash tools/round_profiles.sh $T "c5:--config c5" "c5p:--config c5 --obs packed" \
    "c5s:--config c5 --rng stream" "c5g:--config c5 --rng seeded" "c2:--config c2"
