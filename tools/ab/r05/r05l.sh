set -u
mkdir -p gpurun_out/r05l
timeout -k 10 800 python3 -u -m pytest tests/test_gpu_mt.py tests/test_gpu_golden128.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05l/pytest.log 2>&1 || { tail -30 gpurun_out/r05l/pytest.log; exit 1; }
tail -1 gpurun_out/r05l/pytest.log
for x in 1 2; do
timeout -k 10 300 python3 bench.py --config c5 --rng seeded --no-cpu-baseline --pmc off > gpurun_out/r05l/c5g.json 2> gpurun_out/r05l/c5g.err || { tail -5 gpurun_out/r05l/c5g.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c5g', round(d['value']/1e6,2), 'M/s', d['ms_per_step'], d['roofline'].get('kernel_ms'))" gpurun_out/r05l/c5g.json
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r05l/kt -o kt -- python3 $R/bench.py --config c5 --rng seeded --steps 100 --warmup 20 --no-cpu-baseline --pmc off > $R/gpurun_out/r05l/kt.log 2>&1 || { tail -5 $R/gpurun_out/r05l/kt.log; exit 1; }
find $R/gpurun_out/r05l/kt -name "*kernel_trace.csv" -delete
