#!/bin/bash
# Round-3 session e: 128-column one-launch statistics defaults: their GPU tests, the build A/B,
# the kernel-trace + PMC passes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=quantizers_amd/csrc/build/tune
TAG=r03e TESTS="tests/test_quant_gpu.py tests/test_guard_band_gpu.py tests/test_awq_golden.py" \
  SKIP_BENCH=1 bash scripts/gpu_session.sh || exit $?
timeout -k 10 400 python scripts/tune_stats.py $T/libqz_base.so $T/libqz_new.so $T/libqz_wmb128.so $T/libqz_wmb512.so \
  $T/libqz_ab768.so $T/libqz_ab2048.so $T/libqz_cpg8.so > gpurun_out/r03e_tune_stats.log 2>&1 \
  || { tail -20 gpurun_out/r03e_tune_stats.log; exit 1; }
tail -8 gpurun_out/r03e_tune_stats.log
TAG=r03e bash scripts/pmc_kernels.sh || exit $?
