export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_nvfp4_gpu.py tests/test_oneshot_gpu.py > gpurun_out/r04x_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r04x_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r04x_bench.log 2>&1 || exit 1
python - <<'PY'
import json
d = json.loads([l for l in open("gpurun_out/r04x_bench.log") if l.startswith('{"metric"')][0])
nv = d["other_configs"]["qwen3_30b_a3b_experts_nvfp4"]
print(json.dumps({"value": d["value"], "frac": d["roofline"]["frac"], "nv_ms": nv["ms"], "nv_frac": nv["frac"],
                  "nv_one_stream": nv["one_stream"]["frac"], "nv_two_pass": nv["two_pass_qz_quantize"]["frac"]}))
PY
