#!/bin/bash
# round 6: PMC + SQ attribution of the C3 step kernel, plane mode against the uint16 form
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}
cd $R
bash tools/profile.sh r06e/planes --config c3 || exit 1
bash tools/profile.sh r06e/u16 --config c3 --board-mode uint16 || exit 1
for v in planes u16; do
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    if 'k_env_step_bits64' in k:
        print(sys.argv[2], k[:60], {kk: (round(vv,1) if isinstance(vv,float) else vv) for kk,vv in (v.get('last_k') or v).items() if kk in ('avg_ns','hbm_read_bytes','hbm_write_bytes','hbm_bytes_per_launch','hbm_GBps','valu_per_wave','salu_per_wave','SQ_WAVES','attribution','SQ_INSTS_LDS','SQ_INSTS_VMEM_RD','SQ_INSTS_VMEM_WR','SQ_WAVE_CYCLES')})
" gpurun_out/r06e/$v/summary.json $v
done
