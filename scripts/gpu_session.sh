#!/bin/bash
# One GPU-box session: selected GPU tests, the bench line, and optionally the rocprofv3 kernel
# trace of the same bench command.  Every GPU step has its own time limit; a failure, crash or
# timeout ends the script (no further GPU step after it).
#   TAG=r03x TESTS="tests/test_x.py" BENCH_ARGS="..." PROFILE=0|1 bash scripts/gpu_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r03}
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 12 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
if [ -n "${TESTS:-}" ]; then
  step pytest_gpu "${TEST_TIMEOUT:-420}" python -u -m pytest ${TESTS} -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread
fi
[ "${SKIP_BENCH:-0}" = 1 ] || step bench "${BENCH_TIMEOUT:-400}" python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-0}" = 1 ]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_${TAG}" -o run -- \
       python3 "$PWD/bench.py" ${BENCH_ARGS:-}
fi
echo "=== done"
