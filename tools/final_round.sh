#!/bin/bash
# End-of-round GPU session (round 4 form), in two parts so each fits one gpurun call:
#   tools/final_round.sh <tag> a   parity tests, the headline bench line, profiles +
#                                  PMC records of C3 and its observation forms
#   tools/final_round.sh <tag> b   C5 (Philox, replay, seeded generator) and C2 profiles
#                                  + PMC records, the C5 wave-cycle attribution, and the
#                                  per-config bench lines (C1, C2, C4, C5 forms)
# Writes gpurun_out/<tag>*; afterwards, on the dev box, tools/keep_profile.py copies the
# judged artifacts (kernel stats, summaries, pmc_*.json records) into profiles/.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-r04z}
P=${2:-a}
cd $R
mkdir -p gpurun_out/$T
if [ "$P" = a ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
      > gpurun_out/$T/pytest.log 2>&1 || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
  tail -3 gpurun_out/$T/pytest.log
  bash tools/profile.sh ${T}_c3 || exit 1
  bash tools/profile.sh ${T}_c3p --obs packed || exit 1
  bash tools/profile.sh ${T}_c3ch --obs channels || exit 1
  bash tools/profile.sh ${T}_c3bf --obs channels --obs-dtype bfloat16 || exit 1
  timeout -k 10 600 python3 bench.py --pmc off > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err \
      || { tail -20 gpurun_out/$T/bench.err; exit 1; }
  cat gpurun_out/$T/bench.json
else
  bash tools/profile.sh ${T}_c5 --config c5 || exit 1
  bash tools/profile.sh ${T}_c5s --config c5 --rng stream || exit 1
  bash tools/profile.sh ${T}_c5g --config c5 --rng seeded || exit 1
  bash tools/profile.sh ${T}_c2 --config c2 || exit 1
  bash tools/profile_sq.sh ${T}_c5sq --config c5 || exit 1
  bash tools/gpu_benches.sh $T "c1:--config c1" "c2:--config c2 --pmc off" "c4:--config c4 --pmc off" \
      "c5:--config c5 --pmc off" "c5s:--config c5 --rng stream --pmc off" \
      "c5g:--config c5 --rng seeded --pmc off" || exit 1
fi
