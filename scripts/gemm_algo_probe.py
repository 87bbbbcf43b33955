"""hipBLASLt algorithms for the AWQ expert-search GEMM (tooling; profiles/r03y_gemm_algo_probe.log).

The expert w3 -> w2 searches run F.linear(x, w2') per expert and grid point: x [T, I] (every
calibration token, moe_calibrate_all_experts), w2' [H, I].  For each shape below this lists the
first N algorithms hipBLASLt's heuristic offers for torch.mm's problem (quantizers_amd
qz_gemm_probe_algos), times each one against torch.mm (interleaved, median of rounds) and says
whether its output equals torch.mm's bit for bit.
usage: python scripts/gemm_algo_probe.py [N]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import _lib  # noqa: E402

SHAPES = {"qwen3_30b_a3b w2 [32768,768]x[2048,768]": (32768, 2048, 768),
          "minimax_m2.1 w2 [16384,1536]x[3072,1536]": (16384, 3072, 1536),
          "qwen3_30b_a3b gate/up [32768,2048]x[768,2048]": (32768, 768, 2048)}
WS = int(os.environ.get("HIPBLASLT_WORKSPACE_SIZE", 76 * 1024)) * 1024


def main(want=16):
    lib = _lib.load()
    P, I64 = ctypes.c_void_p, ctypes.c_int64
    lib.qz_gemm_probe_algos.argtypes = [I64, I64, I64, ctypes.c_size_t, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
    lib.qz_gemm_probe_run.argtypes = [ctypes.c_int32, P, P, P, P, ctypes.c_size_t, P]
    dev = torch.device("cuda:0")
    ws = torch.empty(WS, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    for name, (m, n, k) in SHAPES.items():
        x = (torch.randn(m, k, device=dev) * 0.5).to(torch.bfloat16)
        ws_ = [(torch.randn(n, k, device=dev) * 0.02).to(torch.bfloat16) for _ in range(4)]
        ref = torch.nn.functional.linear(x, ws_[0])
        cnt = ctypes.c_int32(0)
        rc = lib.qz_gemm_probe_algos(m, n, k, WS, want, ctypes.byref(cnt))
        assert rc == 0, rc
        out = torch.empty(m, n, dtype=torch.bfloat16, device=dev)
        runs = {"torch": lambda i: torch.nn.functional.linear(x, ws_[i % 4], out=None)}
        same = {}
        for a in range(cnt.value):
            rc = lib.qz_gemm_probe_run(a, x.data_ptr(), ws_[0].data_ptr(), out.data_ptr(), ws.data_ptr(), WS, st.cuda_stream)
            if rc:
                same[a] = None
                continue
            same[a] = bool(torch.equal(out, ref))
            runs[a] = (lambda i, a=a: lib.qz_gemm_probe_run(a, x.data_ptr(), ws_[i % 4].data_ptr(), out.data_ptr(),
                                                            ws.data_ptr(), WS, st.cuda_stream))
        times = {key: [] for key in runs}
        for _ in range(5):
            for key, fn in runs.items():
                for i in range(3):
                    fn(i)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(20):
                    fn(i)
                e1.record()
                torch.cuda.synchronize()
                times[key].append(e0.elapsed_time(e1) / 20 * 1e3)
        flop = 2 * m * n * k
        print(f"== {name}: {cnt.value} algorithms", flush=True)
        for key in runs:
            t = sorted(times[key])[len(times[key]) // 2]
            print(f"  {str(key):6s} {t:8.1f} us  {flop / t / 1e6:7.1f} TFLOP/s  bits==torch: "
                  f"{'-' if key == 'torch' else same[key]}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 16)
