#!/bin/bash
# GPU parity tests only (one process), optional -k filter: tools/gpu_tests.sh [expr]
set -u
mkdir -p gpurun_out/t
if [ $# -gt 0 ]; then
  timeout -k 10 900 python3 -m pytest tests -m gpu -x -q -k "$1" > gpurun_out/t/pytest.log 2>&1; rc=$?
else
  timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/t/pytest.log 2>&1; rc=$?
fi
tail -40 gpurun_out/t/pytest.log
exit $rc
