#!/bin/bash
# 128x128 start-board source A/B: parity of the LDS-DMA pool variant, then C5 rounds.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd $R
mkdir -p gpurun_out/ab128
SAFELIFE_HIP_LIB=$R/safelife-k2_amd/build/variants/b_lds.so timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread \
  -k "128 or tiny_batches" > gpurun_out/ab128/pytest.log 2>&1 || { tail -30 gpurun_out/ab128/pytest.log; exit 1; }
tail -1 gpurun_out/ab128/pytest.log
timeout -k 10 600 python3 tools/bench_variants.py 2 --config c5 > gpurun_out/ab128/c5.log 2>&1 || { tail gpurun_out/ab128/c5.log; exit 1; }
tail -3 gpurun_out/ab128/c5.log
