#!/bin/bash
# A/B of the AWQ statistics kernels' chunking (build variants under quantizers_amd/csrc/build/tune),
# interleaved rounds of scripts/kernel_driver.py with QUANTIZERS_AMD_LIB pointing at each variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in 1 2 3; do
  for lib in quantizers_amd/csrc/build/tune/libqz_*.so; do
    out=$(QUANTIZERS_AMD_LIB=$PWD/$lib timeout -k 10 120 python3 scripts/kernel_driver.py 30 2>&1) || { echo "$out" | tail -3; exit 1; }
    echo "round $r $(basename $lib): $(echo "$out" | grep -E 'absmean|weight_mean' | tr -s ' ' | tr '\n' ' ')"
  done
done
