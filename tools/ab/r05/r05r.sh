set -u
T=r05r
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_regime.py tests/test_gpu_mt.py tests/test_gpu_golden128.py -x -q --timeout 300 --timeout-method thread -k "stream or replay or seeded or golden or 128 or fill" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for rep in 1 2; do
  bash tools/ab_run.sh $T "--config c5 --rng stream" head cur || exit 1
  bash tools/ab_run.sh ${T}g "--config c5 --rng seeded" head cur || exit 1
done
