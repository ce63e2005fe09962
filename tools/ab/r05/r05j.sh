set -u
mkdir -p gpurun_out/r05j
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mt.py -x -q --timeout 300 --timeout-method thread -k "fill or shards or seeded_replay" > gpurun_out/r05j/pytest.log 2>&1 || { tail -30 gpurun_out/r05j/pytest.log; exit 1; }
tail -1 gpurun_out/r05j/pytest.log
for rep in 1 2; do
for r in 420 840 1680 3360; do
  SAFELIFE_MT_ROUNDS=$r timeout -k 10 300 python3 bench.py --config c5 --rng seeded --no-cpu-baseline --pmc off > gpurun_out/r05j/r$r.json 2> gpurun_out/r05j/r$r.err || { echo "r$r failed"; tail -5 gpurun_out/r05j/r$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', d['ms_per_step'], d['roofline'].get('kernel_ms'))" gpurun_out/r05j/r$r.json rounds$r
done
done
