set -u
mkdir -p gpurun_out/r05i
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05i/kt -o kt -- python3 $R/bench.py --config c5 --rng seeded --steps 100 --warmup 20 --no-cpu-baseline --pmc off > $R/gpurun_out/r05i/kt.log 2>&1 || { tail -5 $R/gpurun_out/r05i/kt.log; exit 1; }
find $R/gpurun_out/r05i/kt -name "*kernel_trace.csv" -delete
tail -1 $R/gpurun_out/r05i/kt.log
