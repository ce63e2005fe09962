#!/bin/bash
# 128x128 parity tests, then an A/B of build/variants on c5
set -u
mkdir -p gpurun_out/t128
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "fast" > gpurun_out/t128/pytest.log 2>&1 || { tail -40 gpurun_out/t128/pytest.log; exit 1; }
tail -4 gpurun_out/t128/pytest.log
bash tools/gpu_ab_cfg.sh c5 ${1:-1}
