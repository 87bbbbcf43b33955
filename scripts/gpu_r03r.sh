#!/bin/bash
# Round-3 session r: the MoE-block grid's reference forward inside the fixed routing (planned
# form) -- GPU tests, MoE / MiniMax CLI runs (phase-timed and plain), a kernel trace of the MoE
# run, and the bench line (its AWQ leg now over 3 layers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_moe_eager.py tests/test_oneshot_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r03r_pytest.log 2>&1 \
  || { tail -30 gpurun_out/r03r_pytest.log; exit 1; }
tail -1 gpurun_out/r03r_pytest.log
M="configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048"
X="configs/minimax-m2.1-awq-mixedprec.yaml configs/models/minimax-m2.1-2layers 8,2048"
QZ_AWQ_PHASE_TIMING=1 TO=300 bash scripts/e2e_cli.sh $M r03r_moe_phases > /dev/null || exit $?
echo "phases: $(grep 'phases so far' gpurun_out/e2e_r03r_moe_phases.log | tail -1 | sed 's/.*(s): //')"
rm -rf /tmp/e2e_out_r03r_moe_phases
for k in 1 2; do
  TO=300 bash scripts/e2e_cli.sh $M r03r_moe_$k > /dev/null || exit $?
  echo "moe: $(grep 'AWQ layer' gpurun_out/e2e_r03r_moe_$k.log | sed 's/.* in //' | tr '\n' ' ')"
  rm -rf /tmp/e2e_out_r03r_moe_$k
done
TO=300 bash scripts/e2e_cli.sh $X r03r_minimax > /dev/null || exit $?
echo "minimax: $(grep 'AWQ layer' gpurun_out/e2e_r03r_minimax.log | sed 's/.* in //' | tr '\n' ' ')"
rm -rf /tmp/e2e_out_r03r_minimax
P=gpurun_out/prof_r03r_moe
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml \
  --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 --output /tmp/r03r_moe \
  > gpurun_out/r03r_moe_trace.log 2>&1 || { tail -20 gpurun_out/r03r_moe_trace.log; exit 1; }
rm -rf /tmp/r03r_moe
python3 scripts/e2e_breakdown.py $P/run_kernel_trace.csv 4 "" \
  "do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 under rocprofv3 --kernel-trace, round-3 build (MoE kernels, direct expert GEMMs, planned reference forward); layer 3's span includes save_compressed" \
  > gpurun_out/r03r_moe_breakdown.txt || exit 1
sed -n 4,10p gpurun_out/r03r_moe_breakdown.txt
timeout -k 10 400 python bench.py > gpurun_out/r03r_bench.log 2>&1 || { tail -20 gpurun_out/r03r_bench.log; exit 1; }
tail -c 300 gpurun_out/r03r_bench.log
