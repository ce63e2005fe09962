#!/bin/bash
# round 6: C5 with packed views (fused, exits prefetched) against the unfused path, and
# the board read after every step (auto -> uint16 kernel; planes -> a sync per read)
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=r06b
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "views_match or board_mode_auto or golden128" > gpurun_out/$T/pytest.log 2>&1 \
    || { tail -40 gpurun_out/$T/pytest.log; exit 1; }
tail -2 gpurun_out/$T/pytest.log
bash tools/gpu_benches.sh $T "c5p:--config c5 --obs packed --no-cpu-baseline --pmc off" \
    "c5p_u16:--config c5 --obs packed --board-mode uint16 --no-cpu-baseline --pmc off" \
    "c5_rb:--config c5 --read-board --no-cpu-baseline --pmc off" \
    "c5_rbp:--config c5 --read-board --board-mode planes --no-cpu-baseline --pmc off" \
    "c5:--config c5 --no-cpu-baseline --pmc off" || exit 1
bash tools/kt.sh $T/c5_rbp --config c5 --read-board --board-mode planes || exit 1
