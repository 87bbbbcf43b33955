#!/bin/bash
# Build tuning variants of the whole HIP library (in-tree, git-ignored, they travel with gpurun);
# QUANTIZERS_AMD_LIB=<variant> makes quantizers_amd load one instead of the default build.
set -e
cd "$(dirname "$0")/../quantizers_amd/csrc"
mkdir -p build/tune
for v in "$@"; do  # each arg: NAME:FLAGS, e.g. u4:-DQZ_UNROLL=4
  name=${v%%:*}; flags=${v#*:}
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $flags -shared \
     -o build/tune/libqz_$name.so qz_quant.hip qz_block.hip qz_awq.hip qz_moe.hip qz_experts.hip qz_norm.hip -ldl &
done
wait
ls -la build/tune
