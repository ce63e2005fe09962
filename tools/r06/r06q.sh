#!/bin/bash
# round 6: the branch-free bit deposit of the bit-ring draw pass -- parity, then C5 seeded A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06q}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_golden128.py tests/test_gpu_mt.py tests/test_gpu_board_planes.py tests/test_gpu_headline.py tests/test_gpu_bench_regime.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/ab_run.sh $T/abg "--config c5 --rng seeded" pro_new dep_new pro_new dep_new || exit 1
SAFELIFE_HIP_LIB=$R/variants/dep_new.so bash tools/kt.sh $T/kt --config c5 --rng seeded || exit 1
