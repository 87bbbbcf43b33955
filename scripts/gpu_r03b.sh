#!/bin/bash
# Round-3 session b: full GPU tests + bench, then the statistics / fake-quant build A/Bs, then
# the ONE bmm fault probe (last: a fault there ends the session).  Any failure stops the chain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
T=quantizers_amd/csrc/build/tune
TAG=r03b TESTS=tests TEST_TIMEOUT=600 bash scripts/gpu_session.sh || exit $?
timeout -k 10 300 python scripts/tune_stats.py $T/libqz_base.so $T/libqz_new.so $T/libqz_wm256.so $T/libqz_wm1024.so \
  $T/libqz_ab512.so $T/libqz_ab2048.so > gpurun_out/r03b_tune_stats.log 2>&1 || { tail -20 gpurun_out/r03b_tune_stats.log; exit 1; }
tail -8 gpurun_out/r03b_tune_stats.log
MODE=awq timeout -k 10 300 python scripts/tune_fast.py $T/libqz_base.so $T/libqz_new.so > gpurun_out/r03b_tune_fq.log 2>&1 \
  || { tail -20 gpurun_out/r03b_tune_fq.log; exit 1; }
tail -8 gpurun_out/r03b_tune_fq.log
[ "${PROBE:-0}" = 1 ] || exit 0  # the probe ran once (profiles/r03b_bmm_probe.log)
timeout -k 10 120 python -u scripts/bmm_fault_probe.py > gpurun_out/r03b_bmm_probe.log 2>&1
echo "probe rc=$?"
tail -20 gpurun_out/r03b_bmm_probe.log
