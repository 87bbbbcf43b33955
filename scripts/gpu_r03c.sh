#!/bin/bash
# Round-3 session c: the statistics / fake-quant GPU tests on the fence-free one-launch
# statistics, the build A/B, then the kernel-trace + PMC passes (scripts/pmc_kernels.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=quantizers_amd/csrc/build/tune
TAG=r03c TESTS="tests/test_quant_gpu.py tests/test_guard_band_gpu.py tests/test_awq_golden.py tests/test_oneshot_gpu.py" \
  SKIP_BENCH=1 bash scripts/gpu_session.sh || exit $?
timeout -k 10 300 python scripts/tune_stats.py $T/libqz_base.so $T/libqz_new.so $T/libqz_wm256.so $T/libqz_wm1024.so \
  $T/libqz_ab512.so $T/libqz_ab2048.so > gpurun_out/r03c_tune_stats.log 2>&1 || { tail -20 gpurun_out/r03c_tune_stats.log; exit 1; }
tail -7 gpurun_out/r03c_tune_stats.log
TAG=r03c bash scripts/pmc_kernels.sh || exit $?
# MoE AWQ phase attribution (synchronised per-phase wall times; diagnostic mode), sequential
# and threaded per-sample calls
for th in 1 4; do
  QZ_CALIB_THREADS=$th QZ_AWQ_PHASE_TIMING=1 TO=400 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-awq-int4.yaml \
    configs/models/qwen3-30b-a3b-4layers 16,2048 r03c_moe_phases_t$th || exit $?
  grep "AWQ phases" gpurun_out/e2e_r03c_moe_phases_t$th.log | tail -1
done
