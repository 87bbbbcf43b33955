"""A/B timing of qz_awq_absmean_accum tuning builds (chunking knobs) on one GPU.
usage: python scripts/tune_absmean.py lib1.so lib2.so ...  (each lib: a full libquantizers_amd build)
Times the two-kernel accumulate over bf16 [16384, 4096] activations (the bench's AWQ a3 case) and
checks every build's sums against the first's (fp32, different chunk order -> rtol 1e-5)."""
import ctypes
import sys

import torch

T, C = 16384, 4096


def main():
    dev = torch.device("cuda:0")
    xs = [torch.randn(T, C, device=dev).to(torch.bfloat16) for _ in range(4)]
    first = None
    for path in sys.argv[1:]:
        lib = ctypes.CDLL(path)
        lib.qz_awq_absmean_workspace_size.restype = ctypes.c_size_t
        lib.qz_awq_absmean_workspace_size.argtypes = [ctypes.c_int64, ctypes.c_int64]
        lib.qz_awq_absmean_accum.restype = ctypes.c_int
        lib.qz_awq_absmean_accum.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
        wsb = lib.qz_awq_absmean_workspace_size(T, C)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        sums = torch.zeros(C, dtype=torch.float32, device=dev)
        st = torch.cuda.current_stream().cuda_stream

        def call(i):
            rc = lib.qz_awq_absmean_accum(xs[i % 4].data_ptr(), T, C, C, sums.data_ptr(), ws.data_ptr(), wsb, st)
            assert rc == 0, rc

        call(0)
        torch.cuda.synchronize()
        chk = sums.clone()
        for i in range(20):
            call(i)
        res = []
        for _ in range(5):
            n = 100
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(n):
                call(i)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) / n * 1e3)
        res.sort()
        if first is None:
            first = chk
        ok = torch.allclose(chk, first, rtol=1e-5, atol=1e-3)
        gbs = T * C * 2 / (res[2] * 1e-6) / 1e9
        print(f"{path.split('/')[-1]:24s} ws={wsb/1e6:6.2f} MB  median {res[2]:7.2f} us  min {res[0]:7.2f}  "
              f"-> {gbs:6.0f} GB/s alg  match={ok}", flush=True)


if __name__ == "__main__":
    main()
