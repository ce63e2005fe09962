#!/bin/bash
# round 6: A/B of the 64x64 plane kernel's store forms (tools/ab/r06_planes64.py), and the
# uint16 form, interleaved on one box
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
for rep in 1 2; do
  bash tools/ab_run.sh r06h "--config c3" p64_base p64_fullrow p64_storeall || exit 1
  SAFELIFE_HIP_LIB=$R/variants/p64_base.so timeout -k 10 300 python3 bench.py --config c3 --board-mode uint16 \
      --no-cpu-baseline --pmc off > gpurun_out/r06h/u16_$rep.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('u16', round(d['value']/1e6,2), 'M/s', d['roofline'].get('kernel_ms'))" gpurun_out/r06h/u16_$rep.json
done
