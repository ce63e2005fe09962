#!/bin/bash
# A/B the variant libraries in build/variants on one config: tools/gpu_ab_cfg.sh <cfg> [rounds]
set -u
mkdir -p gpurun_out/ab
timeout -k 10 900 python3 tools/bench_variants.py ${2:-1} --config $1 > gpurun_out/ab/variants_$1.log 2>&1; rc=$?
cat gpurun_out/ab/variants_$1.log
exit $rc
