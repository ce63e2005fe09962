set -u
mkdir -p gpurun_out/r01b
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/r01b/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/r01b/pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python3 tools/bench_variants.py 1 > gpurun_out/r01b/variants.log 2>&1; rc=$?
cat gpurun_out/r01b/variants.log
exit $rc
