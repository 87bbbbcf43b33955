#!/bin/bash
# Round-3 session o: qz_expert_gemms (grid forwards only, calls serialised, per-problem
# verification) -- GPU tests, then MoE and MiniMax CLI runs with it on and off (phase-timed and
# plain), and a kernel trace of the MoE run for the busy-fraction breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
QZ_EXPERT_GEMMS_DEBUG=1 timeout -k 10 500 python -u -m pytest tests/test_moe_eager.py tests/test_oneshot_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 150 --timeout-method thread \
  -k "gemms or combine or silu or fused or graph or moe or minimax or planned or fixed or knob" \
  > gpurun_out/r03o_pytest.log 2>&1 || { tail -30 gpurun_out/r03o_pytest.log; exit 1; }
tail -2 gpurun_out/r03o_pytest.log
M="configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048"
X="configs/minimax-m2.1-awq-mixedprec.yaml configs/models/minimax-m2.1-2layers 8,2048"
for D in 1 0; do
  T=r03o_moe_direct${D}_phases
  QZ_DIRECT_EXPERT_GEMMS=$D QZ_AWQ_PHASE_TIMING=1 TO=300 bash scripts/e2e_cli.sh $M $T > /dev/null || exit $?
  echo "direct=$D: $(grep 'phases so far' gpurun_out/e2e_$T.log | tail -1 | sed 's/.*(s): //')"
  rm -rf /tmp/e2e_out_$T
done
for D in 1 0 1 0; do
  T=r03o_moe_direct$D
  QZ_DIRECT_EXPERT_GEMMS=$D TO=300 bash scripts/e2e_cli.sh $M $T > /dev/null || exit $?
  echo "moe direct=$D: $(grep 'AWQ layer' gpurun_out/e2e_$T.log | sed 's/.* in //' | tr '\n' ' ')"
  rm -rf /tmp/e2e_out_$T
  T=r03o_minimax_direct$D
  QZ_DIRECT_EXPERT_GEMMS=$D TO=300 bash scripts/e2e_cli.sh $X $T > /dev/null || exit $?
  echo "minimax direct=$D: $(grep 'AWQ layer' gpurun_out/e2e_$T.log | sed 's/.* in //' | tr '\n' ' ')"
  rm -rf /tmp/e2e_out_$T
done
P=gpurun_out/prof_r03o_moe
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml \
  --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 --output /tmp/r03o_moe \
  > gpurun_out/r03o_moe_trace.log 2>&1 || { tail -20 gpurun_out/r03o_moe_trace.log; exit 1; }
rm -rf /tmp/r03o_moe
python3 scripts/e2e_breakdown.py $P/run_kernel_trace.csv 4 "" \
  "do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 under rocprofv3 --kernel-trace, round-3 build (qz_moe_combine, qz_moe_silu_mul, qz_expert_gemms in the grid forwards); layer 3's span includes save_compressed" \
  > gpurun_out/r03o_moe_breakdown.txt || exit 1
head -16 gpurun_out/r03o_moe_breakdown.txt
