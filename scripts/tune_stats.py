"""Interleaved A/B of the AWQ statistics kernels (a3 absmean, a4 w_mean) across library builds.
usage: python scripts/tune_stats.py lib1.so lib2.so ...  (each: a full libquantizers_amd build)

Per round and build: 100 back-to-back calls (rotating 4 activation / 12 weight copies, all beyond
the Infinity Cache together), HIP events / 100 -> us per call (both stages).  Rounds interleave
the builds; the median over rounds is printed.  Every build's sums are checked against the first
build's: bit-equal when the reduction tree is the same, else to rtol 1e-5 (f32) / 1e-12 (f64)."""
import ctypes
import os
import sys

import torch

# operand shapes: ABS=TxC (absmean activations), WM=RxC (w_mean weight); defaults: the round-3 pair
T, C = (int(v) for v in os.environ.get("ABS", "16384x4096").split("x"))
R, WC = (int(v) for v in os.environ.get("WM", "11008x4096").split("x"))
G = 128
P = ctypes.c_void_p
I64 = ctypes.c_int64


def bind(path):
    lib = ctypes.CDLL(path)
    lib.qz_awq_absmean_workspace_size.restype = ctypes.c_size_t
    lib.qz_awq_absmean_workspace_size.argtypes = [I64, I64]
    lib.qz_awq_absmean_accum.argtypes = [P, I64, I64, I64, P, P, ctypes.c_size_t, P]
    lib.qz_awq_weight_mean_workspace_size.restype = ctypes.c_size_t
    lib.qz_awq_weight_mean_workspace_size.argtypes = [I64, I64, ctypes.c_int32]
    lib.qz_awq_weight_mean_accum.argtypes = [P, I64, I64, I64, ctypes.c_int32, P, P, ctypes.c_size_t, P]
    return lib


def main():
    dev = torch.device("cuda:0")
    xs = [torch.randn(T, C, device=dev).to(torch.bfloat16) for _ in range(4)]
    ws = [(torch.randn(R, WC, device=dev) * 0.02).to(torch.bfloat16) for _ in range(12)]
    st = torch.cuda.current_stream().cuda_stream
    builds = []
    for path in sys.argv[1:]:
        lib = bind(path)
        na = lib.qz_awq_absmean_workspace_size(T, C)
        nw = lib.qz_awq_weight_mean_workspace_size(R, WC, G)
        b = {"name": path.split("/")[-1], "lib": lib, "wa": torch.zeros(na, dtype=torch.uint8, device=dev),
             "ww": torch.zeros(nw, dtype=torch.uint8, device=dev),
             "sa": torch.zeros(C, dtype=torch.float32, device=dev),
             "sw": torch.zeros(WC, dtype=torch.float64, device=dev), "ta": [], "tw": []}

        def absmean(i, b=b):
            rc = b["lib"].qz_awq_absmean_accum(xs[i % 4].data_ptr(), T, C, C, b["sa"].data_ptr(), b["wa"].data_ptr(),
                                               b["wa"].numel(), st)
            assert rc == 0, rc

        def wmean(i, b=b):
            rc = b["lib"].qz_awq_weight_mean_accum(ws[i % 12].data_ptr(), R, WC, WC, G, b["sw"].data_ptr(),
                                                   b["ww"].data_ptr(), b["ww"].numel(), st)
            assert rc == 0, rc
        b["absmean"], b["wmean"] = absmean, wmean
        b["sa"].zero_(); b["sw"].zero_()
        absmean(0); wmean(0)
        torch.cuda.synchronize()
        b["chk"] = (b["sa"].clone(), b["sw"].clone())
        builds.append(b)
    ref = builds[0]["chk"]
    for b in builds:
        a, w = b["chk"]
        b["eq"] = (torch.equal(a, ref[0]), torch.equal(w, ref[1]))
        b["close"] = (torch.allclose(a, ref[0], rtol=1e-5, atol=1e-3), torch.allclose(w, ref[1], rtol=1e-12, atol=0))
    for rnd in range(7):
        for b in builds:
            for key, tk in (("absmean", "ta"), ("wmean", "tw")):
                fn = b[key]
                for i in range(10):
                    fn(i)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for i in range(100):
                    fn(i)
                e1.record()
                torch.cuda.synchronize()
                b[tk].append(e0.elapsed_time(e1) / 100 * 1e3)
        print(f"round {rnd} done", flush=True)
    for b in builds:
        ta, tw = sorted(b["ta"]), sorted(b["tw"])
        ma, mw = ta[len(ta) // 2], tw[len(tw) // 2]
        print(f"{b['name']:28s} absmean {ma:7.2f} us ({T * C * 2 / ma / 1e3:6.0f} GB/s)  "
              f"w_mean {mw:7.2f} us ({R * WC * 2 / mw / 1e3:6.0f} GB/s)  "
              f"bit-equal (a, w)={b['eq']} close={b['close']}  ws={b['wa'].numel() / 1e6:.2f}/{b['ww'].numel() / 1e6:.2f} MB",
              flush=True)


if __name__ == "__main__":
    main()
