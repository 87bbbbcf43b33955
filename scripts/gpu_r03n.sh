#!/bin/bash
# Round-3 session n: qz_expert_gemms with per-problem verification, and routed (calibration /
# propagation) MoE forwards through the planned form -- GPU tests, MoE CLI A/B with per-phase
# timing (default / QZ_PLANNED_CALLS=0 / QZ_DIRECT_EXPERT_GEMMS=0), plain MoE and MiniMax CLI
# runs, and a kernel trace of the MoE run for the busy-fraction breakdown.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
QZ_EXPERT_GEMMS_DEBUG=1 timeout -k 10 500 python -u -m pytest tests/test_moe_eager.py tests/test_oneshot_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 150 --timeout-method thread \
  -k "gemms or combine or silu or fused or graph or moe or minimax or planned or fixed or knob" \
  > gpurun_out/r03n_pytest.log 2>&1 || { tail -30 gpurun_out/r03n_pytest.log; exit 1; }
tail -2 gpurun_out/r03n_pytest.log
M="configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048"
for V in default QZ_PLANNED_CALLS=0 QZ_DIRECT_EXPERT_GEMMS=0; do
  T=r03n_moe_${V%%=*}
  env $([ $V = default ] || echo $V) QZ_AWQ_PHASE_TIMING=1 TO=300 bash scripts/e2e_cli.sh $M $T > /dev/null || exit $?
  echo "$V: $(grep 'phases so far' gpurun_out/e2e_$T.log | tail -1 | sed 's/.*(s): //')"
  grep "AWQ layer" gpurun_out/e2e_$T.log | sed 's/.*AWQ/  AWQ/'
  rm -rf /tmp/e2e_out_$T
done
TO=300 bash scripts/e2e_cli.sh configs/minimax-m2.1-awq-mixedprec.yaml configs/models/minimax-m2.1-2layers 8,2048 r03n_minimax || exit $?
rm -rf /tmp/e2e_out_r03n_minimax
TO=300 bash scripts/e2e_cli.sh $M r03n_moe_plain || exit $?
rm -rf /tmp/e2e_out_r03n_moe_plain
P=gpurun_out/prof_r03n_moe
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml \
  --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 --output /tmp/r03n_moe \
  > gpurun_out/r03n_moe_trace.log 2>&1 || { tail -20 gpurun_out/r03n_moe_trace.log; exit 1; }
rm -rf /tmp/r03n_moe
python3 scripts/e2e_breakdown.py $P/run_kernel_trace.csv 4 "" \
  "do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 under rocprofv3 --kernel-trace, round-3 build (qz_moe_combine, qz_moe_silu_mul, qz_expert_gemms, planned routed forwards); layer 3's span includes save_compressed" \
  > gpurun_out/r03n_moe_breakdown.txt || exit 1
head -16 gpurun_out/r03n_moe_breakdown.txt
