#!/bin/bash
# Round-3 session d: statistics GPU tests on the two-level one-launch reduction, the build A/B,
# then the kernel-trace + PMC passes (scripts/pmc_kernels.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=quantizers_amd/csrc/build/tune
TAG=r03d TESTS="tests/test_quant_gpu.py tests/test_guard_band_gpu.py tests/test_awq_golden.py" \
  SKIP_BENCH=1 bash scripts/gpu_session.sh || exit $?
timeout -k 10 400 python scripts/tune_stats.py $T/libqz_base.so $T/libqz_new.so $T/libqz_wmb512.so $T/libqz_wmpp0.so \
  $T/libqz_wmnb8.so $T/libqz_abs256.so $T/libqz_cpg16.so $T/libqz_wm128.so > gpurun_out/r03d_tune_stats.log 2>&1 \
  || { tail -20 gpurun_out/r03d_tune_stats.log; exit 1; }
tail -9 gpurun_out/r03d_tune_stats.log
TAG=r03d bash scripts/pmc_kernels.sh || exit $?
