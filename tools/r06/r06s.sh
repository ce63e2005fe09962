#!/bin/bash
# round 6: C5 seeded kernel timeline (start/end of every kernel, both streams)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06s}
mkdir -p $R/gpurun_out/$T
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$T/tr -o tr -- \
    python3 $R/bench.py --config c5 --rng seeded --steps 30 --warmup 10 --no-cpu-baseline --pmc off \
    > $R/gpurun_out/$T/tr.log 2>&1
