set -u
mkdir -p gpurun_out/r04d
timeout -k 10 1000 python -u -m pytest tests/test_gpu_mt.py tests/test_gpu_dropin.py tests/test_gpu_parity.py tests/test_gpu_headline.py -k "mt or fused or g2 or seed or obs or dropin or save or view or setter or state_dict or bench_regime" -x -v --timeout 400 --timeout-method thread > gpurun_out/r04d/pytest.log 2>&1
tail -5 gpurun_out/r04d/pytest.log
bash tools/gpu_benches.sh r04d "c3:--no-cpu-baseline --pmc off" "c3p:--obs packed --no-cpu-baseline --pmc off" "c3ch:--obs channels --no-cpu-baseline --pmc off" "c5g:--config c5 --rng seeded --no-cpu-baseline --pmc off" || exit 1
bash tools/kt.sh r04d_c5g_kt --config c5 --rng seeded || exit 1
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r04d/valu -o valu -- $GRAFT_REPO_ROOT/tools/_bin/valutest > $GRAFT_REPO_ROOT/gpurun_out/r04d/valu.log 2>&1
cat $GRAFT_REPO_ROOT/gpurun_out/r04d/valu.log | grep waves
