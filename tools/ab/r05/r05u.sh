set -u
T=r05u
mkdir -p gpurun_out/$T
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_board_planes.py -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/pytest_bp.log 2>&1 || { tail -40 gpurun_out/$T/pytest_bp.log; exit 1; }
tail -5 gpurun_out/$T/pytest_bp.log
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_headline.py tests/test_gpu_bench_regime.py tests/test_gpu_golden128.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "128 or c5 or C5 or pools2 or pools3 or nav" > gpurun_out/$T/pytest_c5.log 2>&1 || { tail -40 gpurun_out/$T/pytest_c5.log; exit 1; }
tail -2 gpurun_out/$T/pytest_c5.log
for rep in 1 2; do
  bash tools/ab_run.sh $T "--config c5" head cur || exit 1
done
