#!/bin/bash
# Round-4 evidence session (one gpurun call): the bench line, its rocprofv3 kernel trace, the
# per-kernel PMC passes (scripts/pmc_kernels.sh) and the headline FETCH/WRITE passes
# (scripts/pmc_headline.sh).  Every GPU step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r04q}
export TMPDIR=/tmp
TESTS="${TESTS:-tests/test_nvfp4_gpu.py}" SKIP_BENCH=0 PROFILE=1 TAG=$TAG bash scripts/gpu_session.sh || exit $?
TAG=$TAG bash scripts/pmc_kernels.sh || exit $?
TAG=$TAG bash scripts/pmc_headline.sh || exit $?
echo evidence done
