set -u
mkdir -p gpurun_out/r05k
for r in 1260 1680 2100 2520; do
  SAFELIFE_MT_ROUNDS=$r timeout -k 10 300 python3 bench.py --config c5 --rng seeded --no-cpu-baseline --pmc off > gpurun_out/r05k/r$r.json 2> gpurun_out/r05k/r$r.err || { echo "r$r failed"; tail -5 gpurun_out/r05k/r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', d['ms_per_step'], d['roofline'].get('kernel_ms'))" gpurun_out/r05k/r$r.json rounds$r
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05k/kt -o kt -- python3 $R/bench.py --config c5 --rng seeded --steps 100 --warmup 20 --no-cpu-baseline --pmc off > $R/gpurun_out/r05k/kt.log 2>&1 || { tail -5 $R/gpurun_out/r05k/kt.log; exit 1; }
find $R/gpurun_out/r05k/kt -name "*kernel_trace.csv" -delete
