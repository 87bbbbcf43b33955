#!/bin/bash
# Two back-to-back bench.py runs on one box (every leg within 1 %), then
# scripts/bench_compare.py over the two lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06e}
for i in 1 2; do
  timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench$i.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench$i.log; exit 1; }
  echo "bench $i done"
done
python scripts/bench_compare.py gpurun_out/${TAG}_bench1.log gpurun_out/${TAG}_bench2.log | tee gpurun_out/${TAG}_bench_compare.txt
