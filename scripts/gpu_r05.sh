#!/bin/bash
# Round-5 GPU session: FP8_BLOCK variant timing (scripts/tune_block.py), the bench line, and
# optionally the per-kernel PMC passes (scripts/pmc_kernels.sh) / the rocprofv3 trace of bench.py.
# Every GPU step has its own time limit; the first failure ends the session.
#   TAG=r05b TUNE="lib1 lib2" TESTS=tests SMOKE=1 PMC=1 PROFILE=1 HPMC=1 bash scripts/gpu_r05.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r05}
export TMPDIR=/tmp
if [ -n "${TUNE:-}" ]; then
  timeout -k 10 420 python -u scripts/tune_block.py $TUNE > gpurun_out/${TAG}_tune_block.log 2>&1 || exit $?
  echo "tune done"
fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 "${TEST_TIMEOUT:-420}" python -u -m pytest ${TESTS} -m gpu -x -v -p no:cacheprovider --timeout 150 \
      --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  echo "tests done"
fi
if [ "${SMOKE:-0}" = 1 ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
  echo "smoke done"
fi
if [ "${SKIP_BENCH:-0}" != 1 ]; then
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > gpurun_out/${TAG}_bench_plain.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_plain.log; exit 1; }
  echo "bench done"
fi
if [ "${PMC:-0}" = 1 ]; then
  TAG=$TAG bash scripts/pmc_kernels.sh || exit $?
fi
if [ "${PROFILE:-0}" = 1 ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_${TAG}" -o run -- \
       python3 "$PWD/bench.py" ${BENCH_ARGS:-} > gpurun_out/${TAG}_rocprof.log 2>&1 || exit $?
  echo "profile done"
fi
if [ "${HPMC:-0}" = 1 ]; then
  TAG=$TAG bash scripts/pmc_headline.sh || exit $?
fi
echo "session done"
