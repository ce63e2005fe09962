set -u
mkdir -p gpurun_out/r05g
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_mt.py tests/test_gpu_golden128.py tests/test_gpu_bench_regime.py tests/test_gpu_stream_fast.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r05g/pytest.log 2>&1 || { tail -30 gpurun_out/r05g/pytest.log; exit 1; }
tail -2 gpurun_out/r05g/pytest.log
bash tools/ab_run.sh r05g "--config c5 --rng seeded" head mj4 mj8 mj16 head mj4 mj8 mj16 && bash tools/ab_run.sh r05g_s "--config c5 --rng stream" head mj4 head mj4
