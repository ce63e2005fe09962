set -u
mkdir -p gpurun_out/r04x
timeout -k 10 600 python -u -m pytest tests/test_gpu_mt.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r04x/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04x/pytest.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_benches.sh r04x "c5g:--config c5 --rng seeded --no-cpu-baseline --pmc off" "c5s:--config c5 --rng stream --no-cpu-baseline --pmc off" || exit 1
bash tools/kt.sh r04x_c5g_kt --config c5 --rng seeded || exit 1
bash tools/ab_run.sh alab "--obs packed --steps 100 --warmup 10" al_base al_aligned al_short al_base al_aligned || exit 1
bash tools/ab_run.sh pfab "--config c5 --rng stream --steps 100 --warmup 10" pf_base pf_first pf_first_b4 pf_base pf_first
