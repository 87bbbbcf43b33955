#!/bin/bash
# Round-6 session: staging / model_free GPU tests, the model_free measurement, the fused GEMM-loss
# prototype probe.  Each GPU step has its own time limit; the first failure ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-r06i}
if [ "${MFTEST:-1}" = 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_staging_gpu.py tests/test_model_free_gpu.py -m gpu -x -v -p no:cacheprovider \
    --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest.log
fi
if [ "${MF:-1}" = 1 ]; then
  TAG=$TAG bash scripts/gpu_r06_mf.sh || exit $?
fi
if [ "${GEMM:-1}" = 1 ]; then
  timeout -k 10 180 python -u scripts/gemm_loss_probe.py > gpurun_out/${TAG}_gemm_probe.log 2>&1 || { tail -30 gpurun_out/${TAG}_gemm_probe.log; exit 1; }
  cat gpurun_out/${TAG}_gemm_probe.log | grep -v amdgpu.ids
fi
