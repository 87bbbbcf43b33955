#!/bin/bash
# Variants of the FP8_BLOCK strip kernel (qz_block.hip) linked with the default build's other
# objects: NAME:FLAGS args, e.g. nb4:-DQZ_BLK_NB=4.  "base" rebuilds qz_quant.hip
# with QZ_BLK_FAST=0 (the round-1 k_tile_fast path) instead.  Output: build/tune/libqz_NAME.so
set -e
cd "$(dirname "$0")/../quantizers_amd/csrc"
make -s ARCH=gfx950 >/dev/null
mkdir -p build/tune
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics"
OTHERS="build/qz_awq.o build/qz_moe.o build/qz_experts.o build/qz_norm.o"
for v in "$@"; do
  name=${v%%:*}; flags=${v#*:}
  (
    if [ "$name" = base ]; then
      $HIPCC -DQZ_BLK_FAST=0 -c qz_quant.hip -o build/tune/q_$name.o
      $HIPCC -shared -o build/tune/libqz_$name.so build/tune/q_$name.o build/qz_block.o $OTHERS -ldl
    else
      $HIPCC $flags -c qz_block.hip -o build/tune/b_$name.o
      $HIPCC -shared -o build/tune/libqz_$name.so build/qz_quant.o build/tune/b_$name.o $OTHERS -ldl
    fi
  ) &
done
wait
ls build/tune/*.so
