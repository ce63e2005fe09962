#!/bin/bash
# round 6: C5 seeded -- generator block length (SAFELIFE_MT_ROUNDS) x wave priority
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06r}
mkdir -p $R/gpurun_out/$T
cd $R
for rep in 1 2; do
  for r in 840 560 420; do
    SAFELIFE_MT_ROUNDS=$r bash tools/ab_run.sh $T/r$r "--config c5 --rng seeded" dep_new mt_prio || exit 1
  done
done
