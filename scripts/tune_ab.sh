#!/bin/bash
# A/B timing of tuning builds on the GPU box (each step time-limited; stops at the first failure).
# usage: bash scripts/tune_ab.sh "<env for run 1>" "<env for run 2>" ... (libs: build/tune/libqz_*.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
LIBS=$(ls quantizers_amd/csrc/build/tune/libqz_*.so)
for e in "$@"; do
  echo "=== $e"
  env $e timeout -k 10 240 python scripts/tune_fast.py $LIBS || exit $?
done
