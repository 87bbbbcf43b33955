#!/bin/bash
# Round-3 session ai: rocprof kernel durations (the per-launch metric) of the per-weight quantize
# launch for workgroup-size / unroll build variants, each its own rocprofv3 --kernel-trace run of
# scripts/kernel_driver.py; medians by scripts/kernel_medians.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=quantizers_amd/csrc/build/tune
for R in 1 2; do
  for v in base blk256 blk64 un1 un4; do
    O=$PWD/gpurun_out/r03ai_${v}_$R
    QUANTIZERS_AMD_LIB=$T/libqz_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- \
      python3 $PWD/scripts/kernel_driver.py 60 > $O.log 2>&1 || { tail -5 $O.log; exit 1; }
    echo "$v round $R: $(python3 scripts/kernel_medians.py $O/run_kernel_trace.csv)"
  done
done
