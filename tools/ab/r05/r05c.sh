set -u
mkdir -p gpurun_out/r05c
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05c/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/r05c/pytest.log; grep -E "FAIL|Error" gpurun_out/r05c/pytest.log | head -20
[ $rc -eq 0 ] || exit $rc
bash tools/ab_run.sh r05c "" head tail head tail && bash tools/ab_run.sh r05c_p "--obs packed" head tail head tail
