#!/bin/bash
# Round-3 session ae: Qwen3-4B AWQ through the CLI with the moved model's host image kept
# (QZ_HOST_COPY=keep, default) or released on a helper thread (release), alternating.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for H in keep release keep release; do
  T=r03ae_$H
  QZ_HOST_COPY=$H TO=300 bash scripts/e2e_cli.sh configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 $T > /dev/null || exit $?
  echo "host copy $H: $(grep -E 'captured|Completed|Saved' gpurun_out/e2e_$T.log | sed 's/.* - //' | tr '\n' ' ')"
  rm -rf /tmp/e2e_out_$T
done
