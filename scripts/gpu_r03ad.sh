#!/bin/bash
# Round-3 session ad: the Qwen3-4B AWQ setup with synchronised diagnostics (model move, per-sample
# layer-0 capture), once plain and once with QZ_AWQ_PHASE_TIMING=1.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for P in 1; do
  QZ_AWQ_PHASE_TIMING=$P TO=300 bash scripts/e2e_cli.sh configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 r03ad_p$P > /dev/null || exit $?
  echo "== phase timing $P"; grep -E "Starting|move|captur|batched call|AWQ layer (0|1|35):|Completed" gpurun_out/e2e_r03ad_p$P.log | sed 's/ - quantizers_amd[^-]*- / /' | cut -c1-250
  rm -rf /tmp/e2e_out_r03ad_p$P
done
