export TMPDIR=/tmp
T=quantizers_amd/csrc/build/tune
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/r04p_pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r04p_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r04p_pytest_gpu.log
for v in nvtab nvsel nvtab nvsel; do QUANTIZERS_AMD_LIB=$T/libqz_$v.so timeout -k 10 300 python -u scripts/nv_probe.py > gpurun_out/r04p_nvprobe_$v.log 2>&1 || exit 1; grep -E "one_launch|experts_nvfp4_fused|dense" gpurun_out/r04p_nvprobe_$v.log | sed "s/^/$v /" | cut -c1-160; done
