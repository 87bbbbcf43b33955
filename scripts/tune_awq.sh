#!/bin/bash
# Variants of the AWQ statistics kernels (qz_awq.hip) with other values of its tuning constants,
# linked with the default build's other objects.  Args: NAME:CONST=VAL[,CONST=VAL...], e.g.
# blk512:QZ_WM1_BLOCKS=512 ("base": unchanged).  Output: build/tune/libqz_NAME.so
set -e
cd "$(dirname "$0")/../quantizers_amd/csrc"
make -s ARCH=gfx950 >/dev/null
mkdir -p build/tune
HIPCC="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -I."
OTHERS="build/qz_quant.o build/qz_block.o build/qz_moe.o build/qz_experts.o build/qz_norm.o"
for v in "$@"; do
  name=${v%%:*}; sets=${v#*:}
  (
    src=build/tune/awq_$name.hip
    cp qz_awq.hip $src
    if [ "$name" != base ]; then
      for kv in ${sets//,/ }; do
        k=${kv%%=*}; val=${kv#*=}
        grep -q "constexpr int $k = " $src || { echo "no constant $k"; exit 1; }
        sed -i "s/constexpr int $k = [^;]*;/constexpr int $k = $val;/" $src
      done
    fi
    $HIPCC -c $src -o build/tune/a_$name.o
    $HIPCC -shared -o build/tune/libqz_$name.so $OTHERS build/tune/a_$name.o -ldl
  ) &
done
wait
ls build/tune/*.so
