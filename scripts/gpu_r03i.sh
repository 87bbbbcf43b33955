#!/bin/bash
# Round-3 session i: MoE-block grid forwards replayed from one HIP graph -- GPU tests (graph vs
# eager bit equality), then the MoE CLI runs with per-phase timing, graphs on and off.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_oneshot_gpu.py tests/test_moe_eager.py -m gpu -x -v -p no:cacheprovider \
  --timeout 150 --timeout-method thread -k "graph or moe or minimax or planned or fixed" > gpurun_out/r03i_pytest.log 2>&1 \
  || { tail -30 gpurun_out/r03i_pytest.log; exit 1; }
tail -3 gpurun_out/r03i_pytest.log
for G in 1 0; do
  QZ_GRID_GRAPHS=$G QZ_AWQ_PHASE_TIMING=1 TO=300 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-awq-int4.yaml \
    configs/models/qwen3-30b-a3b-4layers 16,2048 r03i_moe_graphs$G || exit $?
  grep -i "phase" gpurun_out/e2e_r03i_moe_graphs$G.log | tail -3
  rm -rf /tmp/e2e_out_r03i_moe_graphs$G
done
QZ_AWQ_PHASE_TIMING=1 TO=300 bash scripts/e2e_cli.sh configs/minimax-m2.1-awq-mixedprec.yaml configs/models/minimax-m2.1-2layers 8,2048 r03i_minimax || exit $?
