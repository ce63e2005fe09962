set -u
mkdir -p gpurun_out/r04e
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r04e/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04e/pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_benches.sh r04e "c3:--no-cpu-baseline --pmc off" "c3p:--obs packed --no-cpu-baseline --pmc off" "c3ch:--obs channels --no-cpu-baseline --pmc off" "c4:--config c4 --no-cpu-baseline --pmc off" || exit 1
bash tools/kt.sh r04e_c3_kt || exit 1
