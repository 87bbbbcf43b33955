#!/bin/bash
# Round-3 session h: GPU busy fraction of the MoE AWQ CLI run (Qwen3-30B-A3B dims, 4 layers) and of
# the dense Qwen3-4B run (4 layers) on the final build: rocprofv3 --kernel-trace, then
# scripts/e2e_breakdown.py.  Outputs: gpurun_out/r03h_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=gpurun_out/prof_r03h_moe
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml \
  --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 --output /tmp/r03h_moe \
  > gpurun_out/r03h_moe_trace.log 2>&1 || { tail -20 gpurun_out/r03h_moe_trace.log; exit 1; }
CSV=$P/run_kernel_trace.csv
python3 scripts/e2e_breakdown.py "$CSV" 4 "" \
  "do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 under rocprofv3 --kernel-trace, round-3 final build (one-launch statistics, 4 concurrent calibration/propagation calls); layer 3's span includes save_compressed" \
  > gpurun_out/r03h_moe_breakdown.txt || exit 1
head -16 gpurun_out/r03h_moe_breakdown.txt
rm -rf /tmp/r03h_moe
P=gpurun_out/prof_r03h_dense
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/awq_e2e.py 4 16 2048 > gpurun_out/r03h_dense_trace.log 2>&1 \
  || { tail -20 gpurun_out/r03h_dense_trace.log; exit 1; }
CSV=$P/run_kernel_trace.csv
python3 scripts/e2e_breakdown.py "$CSV" 4 > gpurun_out/r03h_dense_breakdown.txt || exit 1
head -12 gpurun_out/r03h_dense_breakdown.txt
rm -rf $P/*/run_kernel_trace.csv.gz 2>/dev/null
true
