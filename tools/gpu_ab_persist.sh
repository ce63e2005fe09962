#!/bin/bash
# A/B of the persistent 64x64 kernel variants (build/variants/*.so): parity subset on
# the persistent variants, then bench rounds without and with packed observations.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
mkdir -p gpurun_out/ab
for v in b_p4 c_p3; do
  SAFELIFE_HIP_LIB=$R/safelife-k2_amd/build/variants/$v.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
    -k "fused_obs or fast_kernel_vs_generic or full_batch_sampled or env_batch_vs_oracle or state_overwrite" > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -30 gpurun_out/ab/pytest_$v.log; exit 1; }
  tail -1 gpurun_out/ab/pytest_$v.log
done
timeout -k 10 600 python3 tools/bench_variants.py 2 > gpurun_out/ab/none.log 2>&1 || { tail gpurun_out/ab/none.log; exit 1; }
tail -4 gpurun_out/ab/none.log
timeout -k 10 600 python3 tools/bench_variants.py 2 --obs packed > gpurun_out/ab/packed.log 2>&1 || { tail gpurun_out/ab/packed.log; exit 1; }
tail -4 gpurun_out/ab/packed.log
