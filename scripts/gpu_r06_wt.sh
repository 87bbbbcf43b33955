#!/bin/bash
# Round-6 write-through-tail A/B session: scripts/wt_gate_ab.py over the
# tuning builds named in LIBS (scripts/tune_fast.sh), under a rocprofv3 kernel trace, then the
# rocprof medians by library and leg (scripts/wt_gate_rocprof.py).  TESTS=1 adds the quantize tests.
#   TAG=r06b LIBS="cur gate none" TESTS=1 bash scripts/gpu_r06_wt.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06b}
L=quantizers_amd/csrc/build/tune
paths=""; for v in ${LIBS:-cur gate none}; do paths="$paths $L/libqz_$v.so"; done
SEQ=$PWD/gpurun_out/$TAG.seq timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/prof_$TAG" -o run -- \
  python3 scripts/wt_gate_ab.py $paths > gpurun_out/${TAG}_ab.log 2>&1 || { tail -30 gpurun_out/${TAG}_ab.log; exit 1; }
python scripts/wt_gate_rocprof.py gpurun_out/prof_$TAG/run_kernel_trace.csv gpurun_out/$TAG.seq >> gpurun_out/${TAG}_ab.log 2>&1
grep -v "^[WE]2026" gpurun_out/${TAG}_ab.log | tail -40
if [ "${TESTS:-0}" = 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_quant_gpu.py -m gpu -x -q -p no:cacheprovider --timeout 150 \
      --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; rc=$?
  tail -3 gpurun_out/${TAG}_pytest.log; exit $rc
fi
