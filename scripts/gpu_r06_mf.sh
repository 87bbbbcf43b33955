#!/bin/bash
# Round-6 model_free_ptq measurement: scripts/model_free_bench.py on the box's
# local disk, then optionally the two-bench comparison (BENCH2=1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06h}
df -h /tmp "$PWD" > gpurun_out/${TAG}_df.txt 2>&1
timeout -k 10 500 python -u scripts/model_free_bench.py ${MF_ARGS:-} > gpurun_out/${TAG}_model_free.log 2>&1 || { tail -30 gpurun_out/${TAG}_model_free.log; exit 1; }
grep -v "^RESULT" gpurun_out/${TAG}_model_free.log | tail -20
if [ "${BENCH2:-0}" = 1 ]; then TAG=$TAG bash scripts/gpu_r06_bench2.sh || exit $?; fi
