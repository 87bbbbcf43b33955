export TMPDIR=/tmp
T=quantizers_amd/csrc/build/tune
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_nvfp4_gpu.py > gpurun_out/r04d_tests.log 2>&1 && \
for v in nvp8w3 nvp6w4 nvp4w4 nvhold; do QUANTIZERS_AMD_LIB=$T/libqz_$v.so timeout -k 10 300 python -u scripts/nv_probe.py > gpurun_out/r04d_nvprobe_$v.log 2>&1 || exit 1; done && \
QUANTIZERS_AMD_LIB=$T/libqz_nvp6w4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nvfp4_gpu.py >> gpurun_out/r04d_tests.log 2>&1 && \
QUANTIZERS_AMD_LIB=$T/libqz_nvp4w4.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_nvfp4_gpu.py >> gpurun_out/r04d_tests.log 2>&1
