#!/bin/bash
# One GPU-box session: parity tests, a short bench, a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a crash/timeout (exit >= 124 or signal) ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r01}
step() {  # step <name> <timeout> <cmd...>
  local name=$1 to=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$to" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"; tail -n 25 "gpurun_out/${TAG}_${name}.log"
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "ABORT after $name (rc=$rc)"; exit $rc; fi
  return 0
}
[ "${SKIP_TESTS:-0}" = 1 ] || step pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider ${PYTEST_ARGS:-}
[ "${SKIP_SMOKE:-0}" = 1 ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[ "${SKIP_BENCH:-0}" = 1 ] || step bench 600 python bench.py ${BENCH_ARGS:-}
if [ "${PROFILE:-1}" = 1 ]; then
  export TMPDIR=/tmp
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_${TAG}" -o run -- \
       python3 "$PWD/bench.py" --profile-only --steps 100 --warmup 10
fi
echo "=== done"
