set -u
mkdir -p gpurun_out/r05m
timeout -k 10 1000 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r05m/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r05m/pytest.log; exit $rc
