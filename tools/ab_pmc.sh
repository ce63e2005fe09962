#!/bin/bash
# PMC profiles of a few builds on one box: tools/ab_pmc.sh <tag> "<name>:<lib or ->:<bench args>" ...
# (lib "-" = the in-tree build).  Each runs tools/profile.sh; prints the step kernels'
# time, VALU / SALU per wave and the wave-cycle split.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; args=${rest#*:}
  if [ "$lib" = "-" ]; then unset SAFELIFE_HIP_LIB; else export SAFELIFE_HIP_LIB=$R/$lib; fi
  bash $R/tools/profile.sh ${TAG}_$name $args > /dev/null || { echo "$name failed"; exit 1; }
  python3 - $R/gpurun_out/${TAG}_$name/summary.json $name <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if "k_env_step" in k or "prologue" in k or "draw" in k or "k_env_action" in k:
        g = lambda key: v.get(key) or v.get("last_" + key) or 0
        print(sys.argv[2], k[:48], "us=%.1f" % (g("avg_ns") / 1e3),
              "valu/w=%.0f salu/w=%.0f" % (v.get("valu_per_wave", 0), v.get("salu_per_wave", 0)),
              "cyc/w=%.0f busy=%.0f wait_any=%.0f wait_inst=%.0f" % tuple(
                  (v.get(c, 0) / max(v.get("SQ_WAVES", 1), 1)) for c in
                  ("SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")),
              "GB=%.2f" % (v.get("hbm_bytes_per_launch", 0) / 1e9))
PY
done
