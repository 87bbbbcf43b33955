export TMPDIR=/tmp
T=quantizers_amd/csrc/build/tune
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_nvfp4_gpu.py > gpurun_out/r04c_tests.log 2>&1 && \
QUANTIZERS_AMD_LIB=$T/libqz_nvpipe.so timeout -k 10 300 python -u scripts/nv_probe.py > gpurun_out/r04c_nvprobe_pipe.log 2>&1 && \
QUANTIZERS_AMD_LIB=$T/libqz_nvnopipe.so timeout -k 10 300 python -u scripts/nv_probe.py > gpurun_out/r04c_nvprobe_nopipe.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_quant_gpu.py -k "absmean or weight_mean" >> gpurun_out/r04c_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/tune_stats.py $T/libqz_reg.so $T/libqz_d8b256.so $T/libqz_d8b256nt.so $T/libqz_d8b512nt.so > gpurun_out/r04c_tune_stats.log 2>&1
