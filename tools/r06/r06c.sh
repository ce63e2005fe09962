#!/bin/bash
# round 6: the 64x64 board in planes -- its pair tests, the 64x64 parity tests, the C3 line
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06c}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_board_planes64.py -x -v --timeout 200 \
    --timeout-method thread > gpurun_out/$T/pytest64.log 2>&1 \
    || { tail -60 gpurun_out/$T/pytest64.log; exit 1; }
tail -3 gpurun_out/$T/pytest64.log
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "headline or bench_regime or parity or dropin or symmetry or stream_fast" \
    > gpurun_out/$T/pytest.log 2>&1 || { tail -60 gpurun_out/$T/pytest.log; exit 1; }
tail -3 gpurun_out/$T/pytest.log
bash tools/gpu_benches.sh $T "c3:--config c3 --no-cpu-baseline --pmc off" \
    "c4:--config c4 --no-cpu-baseline --pmc off" || exit 1
bash tools/kt.sh $T/c3 --config c3 || exit 1
