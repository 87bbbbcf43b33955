#!/bin/bash
# One GPU-box session (round 2): parity tests, the default bench line, and the rocprofv3 kernel
# trace of the same bench command.  Every GPU step has its own time limit; a crash / timeout
# (exit >= 124 or a signal) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r02a}
export TMPDIR=/tmp
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 15 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ne 0 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 420 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS:-}
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 300 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  step rocprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_${TAG}" -o run -- \
       python3 "$PWD/bench.py" ${BENCH_ARGS:-}
fi
echo "=== done"
