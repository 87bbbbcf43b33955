#!/bin/bash
# Round-3 session j: kernel trace of the MoE CLI run with the MoE-block grid forwards replayed
# from a HIP graph (QZ_GRID_GRAPHS=1), with per-phase timing, to see where the replays' time goes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
P=gpurun_out/prof_r03j_moe
QZ_GRID_GRAPHS=1 QZ_AWQ_PHASE_TIMING=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$P" -o run -- \
  python3 -u scripts/do_oneshot.py --config configs/qwen3-30b-a3b-awq-int4.yaml \
  --random-init configs/models/qwen3-30b-a3b-4layers --calib-random 16,2048 --output /tmp/r03j_moe \
  > gpurun_out/r03j_moe_trace.log 2>&1 || { tail -20 gpurun_out/r03j_moe_trace.log; exit 1; }
grep -E "AWQ layer|phases" gpurun_out/r03j_moe_trace.log | tail -6
rm -rf /tmp/r03j_moe
