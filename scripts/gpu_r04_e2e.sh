#!/bin/bash
# Round-4 end-to-end CLI runs on the final tree (random-init public dims, one GPU).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04q}
TO=300 bash scripts/e2e_cli.sh configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 ${TAG}_qwen3_4b || exit $?
TO=300 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048 ${TAG}_qwen3_30b_a3b_4layers || exit $?
TO=300 bash scripts/e2e_cli.sh configs/minimax-m2.1-awq-mixedprec.yaml configs/models/minimax-m2.1-2layers 8,2048 ${TAG}_minimax_2layers || exit $?
TO=300 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-nvfp4.yaml configs/models/qwen3-30b-a3b-4layers 4,512 ${TAG}_qwen3_30b_a3b_nvfp4_4layers || exit $?
echo e2e done
