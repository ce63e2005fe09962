set -u
mkdir -p gpurun_out/ab
timeout -k 10 900 python3 tools/bench_variants.py 2 > gpurun_out/ab/variants.log 2>&1; rc=$?
cat gpurun_out/ab/variants.log
exit $rc
