export TMPDIR=/tmp
T=quantizers_amd/csrc/build/tune
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_nvfp4_gpu.py > gpurun_out/r04b_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_quant_gpu.py -k "nvfp4 or tensor_group or absmean or weight_mean" >> gpurun_out/r04b_tests.log 2>&1 && \
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_eager.py >> gpurun_out/r04b_tests.log 2>&1 && \
timeout -k 10 300 python -u scripts/nv_probe.py > gpurun_out/r04b_nvprobe.log 2>&1 && \
timeout -k 10 300 python -u scripts/tune_stats.py $T/libqz_reg.so $T/libqz_d8b256.so $T/libqz_d8b512.so $T/libqz_d4b512.so $T/libqz_d8b256nt.so $T/libqz_d16b256.so > gpurun_out/r04b_tune_stats.log 2>&1 && \
MODE=awq timeout -k 10 300 python -u scripts/tune_fast.py $T/libqz_fqbase.so $T/libqz_fqldnt.so $T/libqz_fqstnt.so $T/libqz_fqr8.so $T/libqz_fqr2.so $T/libqz_fqb256.so > gpurun_out/r04b_tune_fq.log 2>&1
