#!/bin/bash
# Round-3 session z: every GPU test on the current build, then the per-kernel rocprof medians and
# PMC counters (scripts/pmc_kernels.sh over scripts/kernel_driver.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  > gpurun_out/r03z_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r03z_pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r03z_pytest_gpu.log
TAG=r03z bash scripts/pmc_kernels.sh || exit $?
