#!/bin/bash
# Round-3 session m: qz_expert_gemms (per-expert hipBLASLt GEMMs issued from C) --
# GPU tests, MoE CLI runs with per-phase timing (direct GEMMs on / off), MiniMax CLI, and a
# kernel trace of the MoE run for the busy-fraction breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
QZ_EXPERT_GEMMS_DEBUG=1 timeout -k 10 500 python -u -m pytest tests/test_moe_eager.py tests/test_oneshot_gpu.py -m gpu -x -v -p no:cacheprovider \
  --timeout 150 --timeout-method thread -k "gemms or combine or silu or fused or graph or moe or minimax or planned or fixed or knob" \
  > gpurun_out/r03m_pytest.log 2>&1 || { tail -30 gpurun_out/r03m_pytest.log; exit 1; }
tail -3 gpurun_out/r03m_pytest.log
for F in 1 0; do
  QZ_DIRECT_EXPERT_GEMMS=$F QZ_AWQ_PHASE_TIMING=1 TO=300 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-awq-int4.yaml \
    configs/models/qwen3-30b-a3b-4layers 16,2048 r03m_moe_direct$F || exit $?
  grep "phases so far" gpurun_out/e2e_r03m_moe_direct$F.log | tail -1
  rm -rf /tmp/e2e_out_r03m_moe_direct$F
done
TO=300 bash scripts/e2e_cli.sh configs/minimax-m2.1-awq-mixedprec.yaml configs/models/minimax-m2.1-2layers 8,2048 r03m_minimax || exit $?
rm -rf /tmp/e2e_out_r03m_minimax
TO=300 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048 r03m_moe_plain || exit $?
rm -rf /tmp/e2e_out_r03m_moe_plain
P=gpurun_out/prof_r03m_moe
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml \
  --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 --output /tmp/r03m_moe \
  > gpurun_out/r03m_moe_trace.log 2>&1 || { tail -20 gpurun_out/r03m_moe_trace.log; exit 1; }
rm -rf /tmp/r03m_moe
python3 scripts/e2e_breakdown.py $P/run_kernel_trace.csv 4 "" \
  "do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 under rocprofv3 --kernel-trace, round-3 build with qz_moe_combine, qz_moe_silu_mul, qz_expert_gemms; layer 3's span includes save_compressed" \
  > gpurun_out/r03m_moe_breakdown.txt || exit 1
head -16 gpurun_out/r03m_moe_breakdown.txt
