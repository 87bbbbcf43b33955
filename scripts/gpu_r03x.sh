#!/bin/bash
# Round-3 session x: w_mean speed-of-light probes (f32 sums / no group max / |w| only; NOT the
# w_mean arithmetic) and workgroup-size variants, interleaved with the default build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=quantizers_amd/csrc/build/tune
timeout -k 10 300 python scripts/tune_stats.py $T/libqz_base.so $T/libqz_p1.so $T/libqz_p2.so $T/libqz_p3.so \
  $T/libqz_wpb16.so > gpurun_out/r03x_tune_stats.log 2>&1 || { tail -20 gpurun_out/r03x_tune_stats.log; exit 1; }
tail -6 gpurun_out/r03x_tune_stats.log
