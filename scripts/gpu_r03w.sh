#!/bin/bash
# Round-3 session w: statistics walk with wave-uniform buffer-load addressing (stats_walk_u) and
# the fake-quant's buffer-descriptor loads / stores: the statistics and fake-quant tests on the
# default build, then interleaved A/Bs of the variant builds (bit checks against the first).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_quant_gpu.py tests/test_awq_golden.py -m gpu -x -v \
  -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/r03w_pytest.log 2>&1 \
  || { tail -30 gpurun_out/r03w_pytest.log; exit 1; }
tail -1 gpurun_out/r03w_pytest.log
T=quantizers_amd/csrc/build/tune
timeout -k 10 400 python scripts/tune_stats.py $T/libqz_old.so $T/libqz_u1.so $T/libqz_u1a4.so $T/libqz_u2a4.so \
  $T/libqz_u2a4b512.so $T/libqz_u1w8.so > gpurun_out/r03w_tune_stats.log 2>&1 \
  || { tail -20 gpurun_out/r03w_tune_stats.log; exit 1; }
tail -6 gpurun_out/r03w_tune_stats.log
MODE=awq timeout -k 10 300 python scripts/tune_fast.py $T/libqz_old.so $T/libqz_u2a4.so $T/libqz_fqr8.so \
  $T/libqz_fqr2.so > gpurun_out/r03w_tune_fq.log 2>&1 || { tail -20 gpurun_out/r03w_tune_fq.log; exit 1; }
tail -8 gpurun_out/r03w_tune_fq.log
