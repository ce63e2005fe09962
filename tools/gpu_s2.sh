set -u
mkdir -p gpurun_out/s2
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "fast128" > gpurun_out/s2/pytest.log 2>&1 || { tail -40 gpurun_out/s2/pytest.log; exit 1; }
tail -5 gpurun_out/s2/pytest.log
timeout -k 10 600 python3 tools/bench_variants.py 1 --config c5 > gpurun_out/s2/variants.log 2>&1; rc=$?
cat gpurun_out/s2/variants.log
exit $rc
