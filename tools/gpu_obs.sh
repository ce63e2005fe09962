#!/bin/bash
# Fused-observation check: focused parity tests, then the c3 bench with and without
# packed observations, and a kernel trace of the observation run.
# tools/gpu_obs.sh <tag>
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${1:-obs}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread \
    -k "fused_obs or fast_kernel_vs_generic or env_batch_vs_oracle or obs_channels" \
    > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --obs packed > $OUT/bench_packed.json 2> $OUT/bench_packed.err || { tail $OUT/bench_packed.err; exit 1; }
cat $OUT/bench_packed.json
timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $OUT/bench_none.json 2> $OUT/bench_none.err || { tail $OUT/bench_none.err; exit 1; }
cat $OUT/bench_none.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o kt -- python3 $R/bench.py --no-cpu-baseline --obs packed --steps 200 --warmup 20 > $OUT/kt.log 2>&1 || { tail $OUT/kt.log; exit 1; }
head -12 $OUT/kt/kt_kernel_stats.csv 2>/dev/null || find $OUT/kt -name "*stats*"
