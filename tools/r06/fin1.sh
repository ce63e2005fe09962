#!/bin/bash
# round 6 final, part 1: the whole GPU suite, smoke(), the default bench line
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
T=${1:-r06fin}
mkdir -p $R/gpurun_out/$T
cd $R
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/$T/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/$T/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/$T/pytest_gpu.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" \
    > gpurun_out/$T/smoke.log 2>&1 || { tail -20 gpurun_out/$T/smoke.log; exit 1; }
tail -1 gpurun_out/$T/smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/$T/bench_default.json 2> gpurun_out/$T/bench_default.err \
    || { tail -20 gpurun_out/$T/bench_default.err; exit 1; }
cat gpurun_out/$T/bench_default.json
