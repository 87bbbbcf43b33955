#!/bin/bash
# Round-3 session w: statistics walk with wave-uniform buffer-load addressing (stats_walk_u):
# ragged-window / fixed-order tests on the default build, then the interleaved A/B of the
# variant builds (bit checks against the first build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py -m gpu -x -v -k "mean or stats or absmean" \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03w_pytest.log 2>&1 \
  || { tail -30 gpurun_out/r03w_pytest.log; exit 1; }
tail -1 gpurun_out/r03w_pytest.log
T=quantizers_amd/csrc/build/tune
timeout -k 10 500 python scripts/tune_stats.py $T/libqz_old.so $T/libqz_u1.so $T/libqz_u1a4.so $T/libqz_u2a4.so \
  $T/libqz_u2a4b512.so $T/libqz_u1w8.so $T/libqz_u2nt.so $T/libqz_old512.so > gpurun_out/r03w_tune_stats.log 2>&1 \
  || { tail -20 gpurun_out/r03w_tune_stats.log; exit 1; }
tail -9 gpurun_out/r03w_tune_stats.log
