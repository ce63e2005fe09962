#!/bin/bash
# round 6 final, part 2: profiles (kernel trace + PMC passes) of C3 and its view forms
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06fin}
cd $R
bash tools/round_profiles.sh $T "c3:--config c3" "c3p:--config c3 --obs packed" \
    "c3ch:--config c3 --obs channels" "c3bf:--config c3 --obs channels --obs-dtype bfloat16"
