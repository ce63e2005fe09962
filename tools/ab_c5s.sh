set -u
cd $GRAFT_REPO_ROOT
for v in r2base r2lds cur; do
  SAFELIFE_HIP_LIB=$GRAFT_REPO_ROOT/variants/$v.so bash tools/kt.sh r03e_$v --config c5 --rng stream || exit 1
  echo "== $v"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_dropin.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r03e_dropin.log 2>&1; tail -3 gpurun_out/r03e_dropin.log
