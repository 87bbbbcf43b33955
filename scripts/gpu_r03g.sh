#!/bin/bash
# Round-3 session g: one more statistics A/B (window width, batch depth, workgroup size).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=quantizers_amd/csrc/build/tune
mkdir -p gpurun_out
timeout -k 10 500 python scripts/tune_stats.py $T/libqz_new.so $T/libqz_a256.so $T/libqz_a256b2k.so $T/libqz_anb4.so \
  $T/libqz_ab512.so $T/libqz_awpb4.so $T/libqz_wnb8.so $T/libqz_wnb2.so > gpurun_out/r03g_tune_stats.log 2>&1 \
  || { tail -20 gpurun_out/r03g_tune_stats.log; exit 1; }
tail -9 gpurun_out/r03g_tune_stats.log
