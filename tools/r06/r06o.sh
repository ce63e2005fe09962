#!/bin/bash
# round 6: the register-resident bit-ring generator -- parity, then C5 seeded A/B
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06o}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mt.py tests/test_gpu_golden128.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/$T/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/ab_run.sh $T/ab "--config c5 --rng seeded" mt_old mt_new mt_old mt_new || exit 1
bash tools/kt.sh $T/kt --config c5 --rng seeded || exit 1
