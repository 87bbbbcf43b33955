#!/bin/bash
# Round-3 session u: qz_rotary128 for apply_rotary_pos_emb (rotary.fused_rotary) --
# GPU tests, Qwen3-4B CLI with QZ_FUSED_ROTARY on / off (alternating), the MoE CLI, and
# the dense 4-layer breakdown under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_rotary.py tests/test_dense_norm.py tests/test_dense_mlp.py tests/test_moe_eager.py tests/test_oneshot_gpu.py -m gpu -x -v \
  -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r03u_pytest.log 2>&1 \
  || { tail -30 gpurun_out/r03u_pytest.log; exit 1; }
tail -1 gpurun_out/r03u_pytest.log
D="configs/qwen3-4b-awq-g128.yaml configs/models/qwen3-4b 16,2048"
for F in 1 0 1 0; do
  T=r03u_dense_fused$F
  QZ_FUSED_ROTARY=$F TO=300 bash scripts/e2e_cli.sh $D $T > /dev/null || exit $?
  echo "dense fused=$F: $(grep -E 'Completed|Saved' gpurun_out/e2e_$T.log | sed 's/.* in //' | tr '\n' ' ') steady $(grep 'AWQ layer' gpurun_out/e2e_$T.log | sed -n '2,36p' | sed 's/.* in //;s/s$//' | awk '{s+=$1} END {printf "%.4f", s/NR}')"
  rm -rf /tmp/e2e_out_$T
done
TO=300 bash scripts/e2e_cli.sh configs/qwen3-30b-a3b-awq-int4.yaml configs/models/qwen3-30b-a3b-4layers 16,2048 r03u_moe > /dev/null || exit $?
echo "moe: $(grep 'AWQ layer' gpurun_out/e2e_r03u_moe.log | sed 's/.* in //' | tr '\n' ' ')"
rm -rf /tmp/e2e_out_r03u_moe
P=gpurun_out/prof_r03u_dense
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/awq_e2e.py 4 16 2048 > gpurun_out/r03u_dense_trace.log 2>&1 \
  || { tail -20 gpurun_out/r03u_dense_trace.log; exit 1; }
python3 scripts/e2e_breakdown.py $P/run_kernel_trace.csv 4 > gpurun_out/r03u_dense_breakdown.txt || exit 1
sed -n 4,20p gpurun_out/r03u_dense_breakdown.txt
