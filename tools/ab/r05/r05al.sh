set -u
T=r05al
mkdir -p gpurun_out/$T
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_board_planes.py tests/test_gpu_parity.py tests/test_gpu_bench_regime.py tests/test_gpu_headline.py tests/test_gpu_golden128.py tests/test_gpu_mt.py -x -q --timeout 300 --timeout-method thread -k "planes or hi_bits or 128 or c5 or C5 or pools3 or pools2 or golden or seeded" > gpurun_out/$T/pytest.log 2>&1 || { tail -30 gpurun_out/$T/pytest.log; exit 1; }
tail -1 gpurun_out/$T/pytest.log
for rep in 1 2; do
  bash tools/ab_run.sh ${T} "--config c5" head plus || exit 1
  bash tools/ab_run.sh ${T}s "--config c5 --rng stream" head plus || exit 1
done
