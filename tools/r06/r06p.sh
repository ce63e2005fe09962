#!/bin/bash
# round 6: the count prologue's edits in one round -- replay parity, then C5 seeded / replay A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06p}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_board_planes.py tests/test_gpu_golden128.py tests/test_gpu_stream_fast.py tests/test_gpu_bench_regime.py tests/test_gpu_headline.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/ab_run.sh $T/abg "--config c5 --rng seeded" pro_old pro_new pro_old pro_new || exit 1
bash tools/ab_run.sh $T/abs "--config c5 --rng stream" pro_old pro_new pro_old pro_new || exit 1
SAFELIFE_HIP_LIB=$R/variants/pro_old.so bash tools/kt.sh $T/kt_old --config c5 --rng seeded || exit 1
SAFELIFE_HIP_LIB=$R/variants/draw_floor.so bash tools/kt.sh $T/kt_floor --config c5 --rng seeded || exit 1
