#!/bin/bash
# round 6: plane kernel v4 (compile-time keep mask, one action path) against v3
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_board_planes64.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/r06i_pytest.log 2>&1 || { tail -30 gpurun_out/r06i_pytest.log; exit 1; }
tail -1 gpurun_out/r06i_pytest.log
for rep in 1 2; do
  bash tools/ab_run.sh r06i "--config c3" p64_base p64_v4 || exit 1
done
