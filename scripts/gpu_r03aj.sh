#!/bin/bash
# Round-3 session aj: Qwen3-4B AWQ through the CLI with the first-call warm-up beside the model
# move (QZ_WARMUP=1, default) and without, alternating; then the oneshot GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in 1 0 1 0; do
  T=r03aj_w$W
  QZ_WARMUP=$W TO=300 bash scripts/e2e_cli.sh configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 $T > /dev/null || exit $?
  echo "warmup $W: $(grep -E 'captured|Completed' gpurun_out/e2e_$T.log | sed 's/.* - //' | tr '\n' ' ')"
  rm -rf /tmp/e2e_out_$T
done
timeout -k 10 500 python -u -m pytest tests/test_oneshot_gpu.py tests/test_cli_gpu.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r03aj_pytest.log 2>&1 || { tail -30 gpurun_out/r03aj_pytest.log; exit 1; }
tail -1 gpurun_out/r03aj_pytest.log
