set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_oneshot_gpu.py -k "stateful or documented" -m gpu > gpurun_out/r02o_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r02o_pytest.log; [ $rc -ne 0 ] && exit $rc
TAG=r02n bash scripts/pmc_headline.sh > gpurun_out/r02n_pmc.log 2>&1 || exit $?
TAG=r02o bash scripts/pmc_kernels.sh > gpurun_out/pmck_r02o.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > gpurun_out/r02o_bench.log 2>&1
rc=$?; tail -c 600 gpurun_out/r02o_bench.log; exit $rc
