#!/bin/bash
# Round-3 session ag: the batched-call check with sample 0 first -- the oneshot GPU tests, then the
# MoE and dense CLI runs (set-up timings logged).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_oneshot_gpu.py tests/test_cli_gpu.py -m gpu -x -v -p no:cacheprovider \
  --timeout 300 --timeout-method thread > gpurun_out/r03ag_pytest.log 2>&1 || { tail -30 gpurun_out/r03ag_pytest.log; exit 1; }
tail -1 gpurun_out/r03ag_pytest.log
for M in "configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048 r03ag_moe" \
         "configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048 r03ag_dense"; do
  set -- $M
  TO=300 bash scripts/e2e_cli.sh $1 $2 $3 $4 > /dev/null || exit $?
  echo "$4: $(grep -E 'captured|batched call|Completed|Saved' gpurun_out/e2e_$4.log | sed 's/.* - //' | tr '\n' ' ')"
  rm -rf /tmp/e2e_out_$4
done
