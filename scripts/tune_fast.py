"""Interleaved A/B timing of library build variants (one process, rounds interleaved).
usage: python scripts/tune_fast.py build/tune/libqz_a.so build/tune/libqz_b.so ..."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import _lib  # noqa: E402

ROWS, COLS = int(os.environ.get("ROWS", 11008)), int(os.environ.get("COLS", 4096))
G = int(os.environ.get("GROUP", 128))
BITS = int(os.environ.get("BITS", 4))
KIND = os.environ.get("KIND", "int")
COPIES = int(os.environ.get("COPIES", 12))
P = ctypes.c_void_p


def load(path):
    lib = ctypes.CDLL(path)
    lib.qz_quantize.argtypes = [P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                ctypes.POINTER(_lib.QzArgs), ctypes.c_int32, P, P, P, P, P, ctypes.c_size_t, P]
    lib.qz_quantize_workspace_size.argtypes = [ctypes.c_int64] * 3 + [ctypes.POINTER(_lib.QzArgs)]
    lib.qz_quantize_workspace_size.restype = ctypes.c_size_t
    return lib


def awq_main(paths, libs):
    """MODE=awq: the AWQ fake-quant Q(W*s)/s (int4 g128) and the in-place column smoothing."""
    dev = torch.device("cuda:0")
    ws = [(torch.randn(ROWS, COLS, device=dev) * 0.02).to(torch.bfloat16) for _ in range(COPIES)]
    s = (torch.rand(COLS, device=dev) + 0.5).float()
    outs = [torch.empty_like(ws[0]) for _ in range(int(os.environ.get("OUTS", 1)))]  # OUTS=4: outputs beyond the MALL
    out = outs[0]
    a = _lib.QzArgs(4, 0, 1, 2, G, 0, 0, 0)
    for lib in libs:
        lib.qz_awq_fake_quant.argtypes = [P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64,
                                          ctypes.c_int64, ctypes.POINTER(_lib.QzArgs), P, P, P, ctypes.c_size_t, P]
        lib.qz_scale_columns.argtypes = [P, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, P, ctypes.c_int32, P]
    n = libs[0].qz_quantize_workspace_size(1, ROWS, COLS, ctypes.byref(a))
    wsp = torch.empty(n + 256, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    sp = P(st.cuda_stream)
    ops = {
        "fake_quant": (lambda lib, i: lib.qz_awq_fake_quant(P(ws[i % COPIES].data_ptr()), 1, ROWS, COLS, COLS,
                                                            ROWS * COLS, ctypes.byref(a), P(s.data_ptr()),
                                                            P(outs[i % len(outs)].data_ptr()), P(wsp.data_ptr()),
                                                            wsp.numel(), sp),
                       ROWS * COLS * 4),
        "scale_columns": (lambda lib, i: lib.qz_scale_columns(P(ws[i % COPIES].data_ptr()), ROWS, COLS, COLS,
                                                              P(s.data_ptr()), i & 1, sp), ROWS * COLS * 4),
    }
    ref = None
    for lib in libs:
        assert ops["fake_quant"][0](lib, 0) == 0
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        elif not torch.equal(ref.view(torch.int16), out.view(torch.int16)):
            print(f"NOTE: {lib._name} fake-quant output differs")
    K = int(os.environ.get("K", 60))
    for name, (fn, nbytes) in ops.items():
        res = {p: [] for p in paths}
        for rnd in range(int(os.environ.get("ROUNDS", 8))):
            for p, lib in zip(paths, libs):
                for i in range(10):
                    fn(lib, i)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for i in range(K):
                    fn(lib, i)
                e1.record(st)
                torch.cuda.synchronize()
                res[p].append(e0.elapsed_time(e1) * 1e3 / K)
        for p in paths:
            v = sorted(res[p])
            print(f"{name:14s} {os.path.basename(p):22s} median {v[len(v)//2]:7.2f} us  min {v[0]:7.2f} us  "
                  f"-> {nbytes / (v[len(v)//2] * 1e-6) / 1e9:7.0f} GB/s alg")


def grouped_main(paths, libs):
    """MODE=grouped: qz_quantize_grouped over K steps (int4 g128), each step its own output set
    (distinct outputs: OUTS=0) or OUTS rotating output sets."""
    dev = torch.device("cuda:0")
    K = int(os.environ.get("K", 100))
    nouts = int(os.environ.get("OUTS", 0)) or K
    ws = [(torch.randn(ROWS, COLS, device=dev) * 0.02).to(torch.bfloat16) for _ in range(COPIES)]
    a = _lib.QzArgs(4, 0, 1, 2, G, 0, 0, 0)
    codes = [torch.empty(ROWS, COLS // 8, dtype=torch.int32, device=dev) for _ in range(nouts)]
    scale = [torch.empty(ROWS, COLS // G, dtype=torch.bfloat16, device=dev) for _ in range(nouts)]
    tab = torch.tensor([[ws[i % COPIES].data_ptr() for i in range(K)], [codes[i % nouts].data_ptr() for i in range(K)],
                        [scale[i % nouts].data_ptr() for i in range(K)], [0] * K], dtype=torch.int64).reshape(-1).to(dev)
    st = torch.cuda.current_stream()
    sp = P(st.cuda_stream)
    for lib in libs:
        lib.qz_quantize_grouped.argtypes = [ctypes.c_int64, P, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.POINTER(_lib.QzArgs), ctypes.c_int32, P]

    def run(lib):
        assert lib.qz_quantize_grouped(K, P(tab.data_ptr()), ROWS, COLS, ctypes.byref(a), 0, sp) == 0

    ref = None
    for lib in libs:
        run(lib)
        torch.cuda.synchronize()
        cur = codes[-1].clone()
        if ref is None:
            ref = cur
        elif not torch.equal(ref, cur):
            print(f"NOTE: {lib._name} output differs")
    res = {p: [] for p in paths}
    for rnd in range(int(os.environ.get("ROUNDS", 6))):
        for p, lib in zip(paths, libs):
            run(lib)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(3):
                run(lib)
            e1.record(st)
            torch.cuda.synchronize()
            res[p].append(e0.elapsed_time(e1) * 1e3 / (3 * K))
    alg = ROWS * COLS * 2 + ROWS * COLS // 2 + ROWS * COLS // G * 2
    for p in paths:
        v = sorted(res[p])
        print(f"grouped K={K} outs={nouts} {os.path.basename(p):22s} median {v[len(v)//2]:7.2f} us/weight  "
              f"min {v[0]:7.2f} -> {alg / (v[len(v)//2] * 1e-6) / 1e9:7.0f} GB/s alg")


def main():
    paths = sys.argv[1:]
    libs = [load(p) for p in paths]
    if os.environ.get("MODE") == "awq":
        return awq_main(paths, libs)
    if os.environ.get("MODE") == "grouped":
        return grouped_main(paths, libs)
    dev = torch.device("cuda:0")
    ws = [(torch.randn(ROWS, COLS, device=dev) * 0.02).to(torch.bfloat16) for _ in range(COPIES)]
    if KIND == "int":
        a = _lib.QzArgs(BITS, 0, 1, 2, G, 0, 0, 0)
        fmt = 0
        codes = torch.empty(ROWS, COLS * BITS // 32, dtype=torch.int32, device=dev)
        scale = torch.empty(ROWS, COLS // G, dtype=torch.bfloat16, device=dev)
    elif KIND == "fp8":
        a = _lib.QzArgs(8, 1, 1, 2, G, 0, 0, 0)
        fmt = 2
        codes = torch.empty(ROWS, COLS, dtype=torch.uint8, device=dev)
        scale = torch.empty(ROWS, COLS // G, dtype=torch.bfloat16, device=dev)
    elif KIND == "fp8block":
        a = _lib.QzArgs(8, 1, 1, 3, 0, 128, 128, 0)
        fmt = 2
        codes = torch.empty(ROWS, COLS, dtype=torch.uint8, device=dev)
        scale = torch.empty(ROWS // 128, COLS // 128, dtype=torch.bfloat16, device=dev)
    else:  # mx
        a = _lib.QzArgs(4, 1, 1, 2, 32, 0, 0, 3)
        fmt = 3
        codes = torch.empty(ROWS, COLS // 2, dtype=torch.uint8, device=dev)
        scale = torch.empty(ROWS, COLS // 32, dtype=torch.uint8, device=dev)
    # OUTS=n: rotate n distinct output sets (step i writes set i % n; 1 = one shared set)
    nouts = int(os.environ.get("OUTS", 1))
    codes_l = [codes] + [torch.empty_like(codes) for _ in range(nouts - 1)]
    scale_l = [scale] + [torch.empty_like(scale) for _ in range(nouts - 1)]
    n = libs[0].qz_quantize_workspace_size(1, ROWS, COLS, ctypes.byref(a))
    wsp = torch.empty(n + 256, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    sp = P(st.cuda_stream)
    ref = None

    def run(lib, i):
        rc = lib.qz_quantize(P(ws[i % COPIES].data_ptr()), 1, ROWS, COLS, COLS, ROWS * COLS, ctypes.byref(a), fmt,
                             P(codes_l[i % nouts].data_ptr()), P(scale_l[i % nouts].data_ptr()), P(0), P(0),
                             P(wsp.data_ptr()), wsp.numel(), sp)
        assert rc == 0, rc

    for lib in libs:  # correctness: every variant gives identical bits
        run(lib, 0)
        torch.cuda.synchronize()
        cur = (codes.clone(), scale.clone())
        if ref is None:
            ref = cur
        else:
            same = torch.equal(ref[0], cur[0]) and torch.equal(ref[1].view(torch.int16), cur[1].view(torch.int16))
            if not same:
                print(f"NOTE: {lib._name} output differs from {paths[0]} (expected only for probe builds)")
    K = int(os.environ.get("K", 60))
    res = {p: [] for p in paths}
    for rnd in range(int(os.environ.get("ROUNDS", 8))):
        for p, lib in zip(paths, libs):
            for i in range(10):
                run(lib, i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for i in range(K):  # back-to-back launches, one event pair around the region
                run(lib, i)
            e1.record(st)
            torch.cuda.synchronize()
            res[p].append(e0.elapsed_time(e1) * 1e3 / K)
    # reference points: torch copy (read+write 2x90 MB) and a read-only sum over one copy
    src = ws[0]
    dst = torch.empty_like(src)
    for name, fn, nbytes in [("torch.copy_ bf16", lambda i: dst.copy_(ws[i % COPIES]), 2 * src.numel() * 2),
                             ("torch.sum (read)", lambda i: ws[i % COPIES].sum(dtype=torch.float32),
                              src.numel() * 2)]:
        for i in range(10):
            fn(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(K):
            fn(i)
        e1.record(st)
        torch.cuda.synchronize()
        d = [e0.elapsed_time(e1) * 1e3 / K] * (K + 1)
        print(f"{name:28s} mean   {d[K//2]:7.2f} us  -> {nbytes / (d[K//2] * 1e-6) / 1e9:7.0f} GB/s")
    alg = ROWS * COLS * 2 + ROWS * COLS * BITS // 8 + ROWS * COLS // G * 2
    if KIND in ("fp8", "fp8block"):
        alg = ROWS * COLS * 3 + (ROWS * COLS // (G if KIND == "fp8" else 16384)) * 2
    for p in paths:
        v = sorted(res[p])
        print(f"{os.path.basename(p):28s} median {v[len(v)//2]:7.2f} us  min {v[0]:7.2f} us  "
              f"-> {alg / (v[len(v)//2] * 1e-6) / 1e9:7.0f} GB/s alg ({KIND})")


if __name__ == "__main__":
    main()
