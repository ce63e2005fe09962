set -u
mkdir -p gpurun_out/r05n
SAFELIFE_HIP_LIB=$PWD/variants/gen64.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_mt.py -x -q --timeout 200 --timeout-method thread -k "fill" > gpurun_out/r05n/pytest.log 2>&1 || { tail -20 gpurun_out/r05n/pytest.log; exit 1; }
tail -1 gpurun_out/r05n/pytest.log
for rep in 1 2; do
for v in gen256 gen128 gen64; do
for r in 840 1680; do
  SAFELIFE_MT_ROUNDS=$r SAFELIFE_HIP_LIB=$PWD/variants/$v.so timeout -k 10 300 python3 bench.py --config c5 --rng seeded --no-cpu-baseline --pmc off > gpurun_out/r05n/$v-$r.json 2> gpurun_out/r05n/$v-$r.err || { echo "$v $r failed"; tail -5 gpurun_out/r05n/$v-$r.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', d['ms_per_step'], d['roofline'].get('kernel_ms'))" gpurun_out/r05n/$v-$r.json $v-$r
done
done
done
