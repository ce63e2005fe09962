set -u
mkdir -p gpurun_out/r04c
timeout -k 10 900 python -u -m pytest tests/test_gpu_mt.py tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "mt or fused or g2 or seed or obs or dropin or save or view or setter or state_dict" -x -v --timeout 300 --timeout-method thread > gpurun_out/r04c/pytest.log 2>&1
tail -5 gpurun_out/r04c/pytest.log
bash tools/gpu_benches.sh r04c "c3ch:--obs channels --no-cpu-baseline --pmc off" "c3bf:--obs channels --obs-dtype bfloat16 --no-cpu-baseline --pmc off" "c5g:--config c5 --rng seeded --no-cpu-baseline --pmc off" || exit 1
bash tools/ab_run.sh r04c_rl "" rl_base rl_list rl_base rl_list || exit 1
bash tools/ab_run.sh r04c_db "--config c5 --rng stream" db_8 db_16 db_24 db_8 db_16 db_24 || exit 1
bash tools/kt.sh r04c_c5g_kt --config c5 --rng seeded || exit 1
SAFELIFE_HIP_LIB=$PWD/variants/rl_list.so timeout -k 10 600 python -u -m pytest tests/test_gpu_headline.py -k "bench_regime and (none or packed)" -x -v --timeout 300 --timeout-method thread > gpurun_out/r04c/pytest_rl.log 2>&1
tail -3 gpurun_out/r04c/pytest_rl.log
bash tools/ab_run.sh r04c_rlp "--obs packed" rl_base rl_list rl_base rl_list || exit 1
(cd /tmp && timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r04c/counters.txt 2>&1) || true
bash tools/profile_sq.sh r04c_c5sq --config c5
