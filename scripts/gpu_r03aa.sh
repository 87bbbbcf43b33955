#!/bin/bash
# Round-3 session aa: MoE AWQ (Qwen3-30B-A3B shape, 4 layers) with 2 / 4 / 8 concurrent
# per-expert GEMM streams in the planned grid forwards (QZ_EXPERT_STREAMS), alternating, with
# the synchronised phase times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp QZ_AWQ_PHASE_TIMING=1
M="configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048"
for S in 4 8 2 4 8 2; do
  T=r03aa_streams$S
  QZ_EXPERT_STREAMS=$S TO=300 bash scripts/e2e_cli.sh $M $T > /dev/null || exit $?
  echo "streams=$S: $(grep 'AWQ layer' gpurun_out/e2e_$T.log | sed 's/.* in //' | tr '\n' ' ') | $(grep 'phases so far' gpurun_out/e2e_$T.log | tail -1 | sed 's/.*(s): //')"
  rm -rf /tmp/e2e_out_$T
done
