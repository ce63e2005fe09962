#!/bin/bash
# Build tuning variants from alternative sl_bits.hip sources into build/variants/.
# Usage: tools/build_src_variants.sh name:path/to/sl_bits.hip:"-DFLAGS" ...
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/safelife-k2_amd/csrc
OUT=$R/safelife-k2_amd/build/variants
mkdir -p $OUT
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -munsafe-fp-atomics -fno-gpu-rdc -ffp-contract=off"
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; src=${rest%%:*}; defs=${rest#*:}
  [ "$defs" = "$rest" ] && defs=""
  tmp=$R/build_v/$name          # two levels below the repo root: ../../include resolves
  mkdir -p $tmp
  cp $C/*.hip $C/*.h $tmp/
  cp $src $tmp/sl_bits.hip
  /opt/rocm/bin/hipcc $FLAGS -DSL_FAST_IMPL=2 $defs $tmp/sl_board.hip $tmp/sl_env.hip $tmp/sl_fast.hip $tmp/sl_bits.hip $tmp/sl_bits128.hip $tmp/sl_bits_small.hip $tmp/sl_rollout.hip -o $OUT/$name.so &
done
wait
ls -la $OUT
