set -u
mkdir -p gpurun_out/r05p
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mt.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05p/pytest_mt.log 2>&1 || { tail -30 gpurun_out/r05p/pytest_mt.log; exit 1; }
tail -1 gpurun_out/r05p/pytest_mt.log
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_headline.py -x -v --timeout 300 --timeout-method thread -k "full_batch_every_env" --durations=5 > gpurun_out/r05p/pytest_fb.log 2>&1 || { tail -30 gpurun_out/r05p/pytest_fb.log; exit 1; }
tail -8 gpurun_out/r05p/pytest_fb.log
for rep in 1 2; do
  bash tools/ab_run.sh r05p "--config c5 --rng seeded" atom cur || exit 1
  SAFELIFE_MT_PRIO=3 bash tools/ab_run.sh r05p_prio "--config c5 --rng seeded" cur || exit 1
done
