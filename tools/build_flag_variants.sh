#!/bin/bash
# Build tuning variants of the whole library with extra -D flags into build/variants/.
# Usage: tools/build_flag_variants.sh name:"-DFLAGS" ...   (old variants are removed)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/safelife-k2_amd/csrc
OUT=$R/safelife-k2_amd/build/variants
mkdir -p $OUT
rm -f $OUT/*.so
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -munsafe-fp-atomics -fno-gpu-rdc -ffp-contract=off"
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  [ "$defs" = "$spec" ] && defs=""
  /opt/rocm/bin/hipcc $FLAGS $defs $C/sl_board.hip $C/sl_env.hip $C/sl_fast.hip $C/sl_bits.hip \
      $C/sl_bits128.hip -o $OUT/$name.so &
done
wait
ls -la $OUT
