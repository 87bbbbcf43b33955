"""Interleaved timing of FP8_BLOCK 128x128 library variants (scripts/tune_block.sh) on the
Qwen3-4B attention shapes of BASELINE.json configs[2], outputs bit-checked against the first
library.  usage: python scripts/tune_block.py build/tune/libqz_a.so build/tune/libqz_b.so ...

Cases: batch launches over [36, r, c] stacks (qz_quantize), per-weight launches (qz_quantize),
grouped launches over a pointer table (qz_quantize_grouped; a library that refuses them --
the round-1 path -- runs qz_quantize_many instead), and the three grouped launches of the
mixed plan's attention half back to back.  HIP events, median over ROUNDS."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import _lib  # noqa: E402

P = ctypes.c_void_p
I64 = ctypes.c_int64
A = ctypes.POINTER(_lib.QzArgs)
ROUNDS = int(os.environ.get("ROUNDS", 7))
B_PER_PARAM = 2 + 1 + 2 / 16384  # read bf16, write e4m3, one bf16 scale per 128x128 block


def load(path):
    lib = ctypes.CDLL(path)
    lib.qz_quantize.argtypes = [P, I64, I64, I64, I64, I64, A, ctypes.c_int32, P, P, P, P, P, ctypes.c_size_t, P]
    lib.qz_quantize_grouped.argtypes = [I64, P, I64, I64, A, ctypes.c_int32, P]
    lib.qz_quantize_many.argtypes = [I64, P, P, P, P, P, I64, I64, I64, I64, I64, A, ctypes.c_int32, P,
                                     ctypes.c_size_t, P]
    return lib


def main(paths):
    libs = [load(p) for p in paths]
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    a = _lib.QzArgs(8, 1, 1, 3, 0, 128, 128, 0)  # FP8_BLOCK
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream()
    sp = P(st.cuda_stream)

    def rnd(*shape):
        return (torch.randn(*shape, device=dev, generator=gen) * 0.02).to(torch.bfloat16)

    def outs(n, r, c):
        return [(torch.empty(r, c, dtype=torch.uint8, device=dev),
                 torch.empty(r // 128, c // 128, dtype=torch.bfloat16, device=dev)) for _ in range(n)]

    cases = []
    # batch launches over stacked layers (the bench's round-4 config-3 leg)
    for name, r, c, copies in (("stack36_1024x2560", 1024, 2560, 3), ("stack36_4096x2560", 4096, 2560, 2)):
        xs = [rnd(36, r, c) for _ in range(copies)]
        o = outs(copies, 36 * r, c)

        def fn(lib, i, xs=xs, o=o, r=r, c=c):
            q, s = o[i % len(o)]
            return lib.qz_quantize(P(xs[i % len(xs)].data_ptr()), 36, r, c, c, r * c, ctypes.byref(a), 2,
                                   P(q.data_ptr()), P(s.data_ptr()), P(0), P(0), P(ws.data_ptr()), ws.numel(), sp)
        cases.append((name, fn, 36 * r * c, 1, lambda o=o: o[0]))
    # per-weight launches and grouped launches over distinct weights (the product plan's shapes)
    groups = {}
    for name, r, c, n in (("kv_1024x2560", 1024, 2560, 72), ("q_4096x2560", 4096, 2560, 36),
                          ("o_2560x4096", 2560, 4096, 36)):
        xs = [rnd(r, c) for _ in range(n)]
        o = outs(n, r, c)
        tab = torch.tensor([[x.data_ptr() for x in xs], [q.data_ptr() for q, _ in o], [s.data_ptr() for _, s in o],
                            [0] * n], dtype=torch.int64).reshape(-1).to(dev)
        wp = (P * n)(*[x.data_ptr() for x in xs])
        qp = (P * n)(*[q.data_ptr() for q, _ in o])
        spp = (P * n)(*[s.data_ptr() for _, s in o])

        def one(lib, i, xs=xs, o=o, r=r, c=c):
            q, s = o[i % len(o)]
            return lib.qz_quantize(P(xs[i % len(xs)].data_ptr()), 1, r, c, c, r * c, ctypes.byref(a), 2,
                                   P(q.data_ptr()), P(s.data_ptr()), P(0), P(0), P(ws.data_ptr()), ws.numel(), sp)

        def grouped(lib, i, n=n, tab=tab, r=r, c=c, wp=wp, qp=qp, spp=spp):
            rc = lib.qz_quantize_grouped(n, P(tab.data_ptr()), r, c, ctypes.byref(a), 2, sp)
            if rc == _lib.QZ_ERR_FORMAT:  # round-1 library: one launch per weight
                rc = lib.qz_quantize_many(n, wp, qp, spp, None, None, 1, r, c, c, r * c, ctypes.byref(a), 2,
                                          P(ws.data_ptr()), ws.numel(), sp)
            return rc
        groups[name] = grouped
        cases.append(("one_" + name, one, r * c, 1, lambda o=o: o[0]))
        cases.append(("grouped_" + name, grouped, n * r * c, 1, lambda o=o: o[-1]))

    def plan(lib, i):  # the attention half of the mixed plan: q, k+v, o grouped launches
        for g in groups.values():
            rc = g(lib, i)
            if rc:
                return rc
        return 0
    cases.append(("plan_attention_q_kv_o", plan, (72 * 1024 + 36 * 4096) * 2560 + 36 * 2560 * 4096, 1,
                  lambda: None))

    for name, fn, params, _, probe in cases:
        ref = None
        for p, lib in zip(paths, libs):
            assert fn(lib, 0) == 0, (name, p)
            torch.cuda.synchronize()
            got = probe()
            if got is not None:
                got = (got[0].clone(), got[1].view(torch.int16).clone())
                if ref is None:
                    ref = got
                elif not (torch.equal(ref[0], got[0]) and torch.equal(ref[1], got[1])):
                    print(f"MISMATCH {name} {os.path.basename(p)}", flush=True)
        k = 40 if params < 1e8 else 10
        res = {p: [] for p in paths}
        for _ in range(ROUNDS):
            for p, lib in zip(paths, libs):
                for i in range(3):
                    fn(lib, i)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for i in range(k):
                    fn(lib, i)
                e1.record(st)
                torch.cuda.synchronize()
                res[p].append(e0.elapsed_time(e1) * 1e3 / k)
        for p in paths:
            v = sorted(res[p])
            med = v[len(v) // 2]
            print(f"{name:26s} {os.path.basename(p):24s} median {med:9.2f} us  min {v[0]:9.2f} us  "
                  f"frac {params * B_PER_PARAM / (med * 1e-6) / 8e12:.3f}", flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
