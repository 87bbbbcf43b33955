#!/bin/bash
# Round-3 evidence session on the final build: every GPU test, smoke, the bench line, the
# rocprofv3 kernel trace of the same bench command, the headline PMC traffic passes, and the
# end-to-end CLI runs (dense / MoE / MiniMax shapes).  Any failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03f}
TAG=$TAG TESTS=tests TEST_TIMEOUT=600 PROFILE=1 bash scripts/gpu_session.sh || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
TAG=$TAG bash scripts/pmc_headline.sh || exit $?
TO=300 bash scripts/e2e_cli.sh configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 ${TAG}_qwen3_4b || exit $?
TO=300 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048 ${TAG}_qwen3_30b_a3b_4layers || exit $?
TO=300 bash scripts/e2e_cli.sh configs/minimax-m2.1-awq-mixedprec.yaml configs/models/minimax-m2.1-2layers 8,2048 ${TAG}_minimax_2layers || exit $?
echo "=== session done"
