set -u
mkdir -p gpurun_out/r05o
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_regime.py tests/test_gpu_headline.py -x -q --timeout 300 --timeout-method thread -k "obs or packed or fused or regime or full_batch" > gpurun_out/r05o/pytest.log 2>&1 || { tail -30 gpurun_out/r05o/pytest.log; exit 1; }
tail -1 gpurun_out/r05o/pytest.log
bash tools/ab_run.sh r05o "--obs packed" pre_dw dw pre_dw dw pre_dw dw
