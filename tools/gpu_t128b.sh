#!/bin/bash
set -u
mkdir -p gpurun_out/t128
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "fast" > gpurun_out/t128/pytest.log 2>&1 || { tail -40 gpurun_out/t128/pytest.log; exit 1; }
tail -2 gpurun_out/t128/pytest.log
timeout -k 10 300 python3 tools/phase_timing128.py safelife-k2_amd/build/variants/t_pf1.so > gpurun_out/t128/phase.txt 2>&1 ; cat gpurun_out/t128/phase.txt
rm -f safelife-k2_amd/build/variants/t_*.so
bash tools/gpu_ab_cfg.sh c5 ${1:-1}
