#!/bin/bash
# round 6: the chains jumps on their own stream -- generator parity, then C5 seeded A/B + timeline
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06v}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mt.py tests/test_gpu_golden128.py tests/test_gpu_stream_fast.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/ab_run.sh $T/abg "--config c5 --rng seeded" nosplit split nosplit split || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/$T/tr -o tr -- \
    python3 $R/bench.py --config c5 --rng seeded --steps 30 --warmup 10 --no-cpu-baseline --pmc off \
    > $R/gpurun_out/$T/tr.log 2>&1
