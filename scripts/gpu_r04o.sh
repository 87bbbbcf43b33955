export TMPDIR=/tmp
T=quantizers_amd/csrc/build/tune
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nvfp4_gpu.py tests/test_quant_gpu.py tests/test_golden.py -k "nvfp4 or tensor_group or fused_experts or small_slices or grouped_dense or larger_than or two_streams or golden" > gpurun_out/r04o_tests.log 2>&1 || { tail -30 gpurun_out/r04o_tests.log; exit 1; }
tail -2 gpurun_out/r04o_tests.log
for v in nvtab nvsel nvtab nvsel; do QUANTIZERS_AMD_LIB=$T/libqz_$v.so timeout -k 10 300 python -u scripts/nv_probe.py > gpurun_out/r04o_nvprobe_$v.log 2>&1 || exit 1; grep -E "one_launch|experts_nvfp4|dense" gpurun_out/r04o_nvprobe_$v.log | sed "s/^/$v /"; done
