#!/bin/bash
# A/B of the bmm guard on the Qwen3-4B AWQ CLI run (alternating, two runs each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for i in 1 2; do for g in 1 0; do
  QZ_BMM_GUARD=$g TO=200 bash scripts/e2e_cli.sh configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 r04s_guard${g}_$i > /dev/null || exit $?
  echo "guard=$g run $i: $(grep -E 'captured|checked in|AWQ layer 0:|Completed' gpurun_out/e2e_r04s_guard${g}_$i.log | sed 's/.*INFO - //' | tr '\n' ' ')"
done; done
