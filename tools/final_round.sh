#!/bin/bash
# End-of-round GPU session: parity tests, the headline bench + profile (tools/gpu_round.sh),
# C5 and C2 profiles, the PMC records of this build, every per-config bench line.
# Usage: tools/final_round.sh <tag>   (writes gpurun_out/<tag>*; run on the GPU box)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
T=${1:-r02f}
cd $R
bash tools/gpu_round.sh $T || exit 1
bash tools/profile.sh ${T}_c5 --config c5 || exit 1
bash tools/profile.sh ${T}_c2 --config c2 || exit 1
python3 tools/keep_profile.py gpurun_out/$T/prof $T --pmc-config c3 > /dev/null || exit 1
python3 tools/keep_profile.py gpurun_out/${T}_c5 ${T}_c5 --pmc-config c5 > /dev/null || exit 1
python3 tools/keep_profile.py gpurun_out/${T}_c2 ${T}_c2 --pmc-config c2 > /dev/null || exit 1
bash tools/gpu_benches.sh $T c2:"--config c2" c5:"--config c5" c4:"--config c4" c3p:"--obs packed" \
    c3s:"--rng stream" c2s:"--config c2 --rng stream" c5s:"--config c5 --rng stream"
