#!/bin/bash
# Round-3 session p: MoE CLI with 4 / 6 / 8 concurrent per-sample calibration / propagation calls
# (QZ_CALIB_THREADS), phase-timed and plain.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
M="configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048"
for N in 4 8 6; do
  T=r03p_moe_threads${N}_phases
  QZ_CALIB_THREADS=$N QZ_AWQ_PHASE_TIMING=1 TO=300 bash scripts/e2e_cli.sh $M $T > /dev/null || exit $?
  echo "threads=$N: $(grep 'phases so far' gpurun_out/e2e_$T.log | tail -1 | sed 's/.*(s): //')"
  rm -rf /tmp/e2e_out_$T
done
for N in 4 8 4 8; do
  T=r03p_moe_threads$N
  QZ_CALIB_THREADS=$N TO=300 bash scripts/e2e_cli.sh $M $T > /dev/null || exit $?
  echo "threads=$N: $(grep 'AWQ layer' gpurun_out/e2e_$T.log | sed 's/.* in //' | tr '\n' ' ')"
  rm -rf /tmp/e2e_out_$T
done
