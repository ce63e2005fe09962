#!/bin/bash
# round 6: kernel traces + PMC of the plane kernels (c3, c3p, c4, c5, c5p, c5s)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
bash tools/round_profiles.sh r06n "c3:--config c3" "c3p:--config c3 --obs packed" \
    "c5:--config c5" "c5p:--config c5 --obs packed" "c5s:--config c5 --rng stream" || exit 1
