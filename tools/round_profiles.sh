#!/bin/bash
# Profiles of the other configs on the GPU box (after tools/gpu_round.sh):
#   tools/round_profiles.sh <tag> "<name>:<bench args>" ...
# Each runs tools/profile.sh into gpurun_out/<tag>_<name>; keep them afterwards, in the
# repo, with tools/keep_profile.py gpurun_out/<tag>_<name> <tag>_<name> --pmc-config <rec>.
# The first failure ends the run.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
cd $R
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  bash tools/profile.sh ${TAG}_$name $args > /dev/null || { echo "$name profile failed"; exit 1; }
  echo "$name profiled"
done
