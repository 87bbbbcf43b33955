export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_nvfp4_gpu.py tests/test_lib_exports.py > gpurun_out/r04k_tests.log 2>&1 || { tail -30 gpurun_out/r04k_tests.log; exit 1; }
tail -3 gpurun_out/r04k_tests.log
timeout -k 10 300 python -u scripts/nv_probe.py > gpurun_out/r04k_nvprobe.log 2>&1 && cat gpurun_out/r04k_nvprobe.log
