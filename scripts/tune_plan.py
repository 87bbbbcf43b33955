"""Interleaved timing of whole-library variants on the bench headline's launch plan: the product's
CompressionPlan over the Qwen3-4B model (int4 g128, 5 grouped launches per step; RECIPE=mixed: the
BASELINE configs[2] mixed recipe instead), replayed through each library's own
qz_quantize_grouped (same device tables, same outputs), outputs bit-checked against the first.
usage: python scripts/tune_plan.py lib_a.so lib_b.so ...   (HIP events, median of ROUNDS x K steps)"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from quantizers_amd import _lib  # noqa: E402
from quantizers_amd.compressor import CompressionPlan, compression_units  # noqa: E402

P = ctypes.c_void_p
I64 = ctypes.c_int64


def main(paths):
    libs = []
    for p in paths:
        lib = ctypes.CDLL(p)
        lib.qz_quantize_grouped.argtypes = [I64, P, I64, I64, ctypes.POINTER(_lib.QzArgs), ctypes.c_int32, P]
        libs.append(lib)
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    recipe = bench.MIXED_RECIPE if os.environ.get("RECIPE") == "mixed" else bench.RECIPE
    model = bench.build_model(dev, recipe)
    plan = CompressionPlan(compression_units(model)[0], dev)
    assert not plan.singles
    calls = [(gq.n, P(gq.table.data_ptr()), gq.rows, gq.cols, gq.ca, gq.out_fmt, gq) for gq, *_ in plan.grouped]
    st = torch.cuda.current_stream()
    sp = P(st.cuda_stream)

    def step(lib, which=None):
        for n, tab, r, c, ca, fmt, _ in (calls if which is None else [calls[which]]):
            rc = lib.qz_quantize_grouped(n, tab, r, c, ctypes.byref(ca), fmt, sp)
            assert rc == 0, rc
    ref = None
    for p, lib in zip(paths, libs):
        step(lib)
        torch.cuda.synchronize()
        got = [torch.cat([o["codes"].reshape(-1).view(torch.uint8) for o in gq.outs] +
                         [o["scale"].reshape(-1).view(torch.uint8) for o in gq.outs]) for *_, gq in calls]
        if ref is None:
            ref = got
        elif not all(torch.equal(a, b) for a, b in zip(ref, got)):
            print(f"MISMATCH {os.path.basename(p)}", flush=True)
    k, rounds = int(os.environ.get("K", 20)), int(os.environ.get("ROUNDS", 9))
    for which in [None] + list(range(len(calls))):
        res = {p: [] for p in paths}
        for _ in range(rounds):
            for p, lib in zip(paths, libs):
                for _ in range(3):
                    step(lib, which)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(k):
                    step(lib, which)
                e1.record(st)
                torch.cuda.synchronize()
                res[p].append(e0.elapsed_time(e1) * 1e3 / k)
        name = "step" if which is None else f"launch {calls[which][6].rows}x{calls[which][6].cols} x{calls[which][0]}"
        for p in paths:
            v = sorted(res[p])
            print(f"{name:26s} {os.path.basename(p):24s} median {v[len(v) // 2]:9.2f} us  min {v[0]:9.2f} us",
                  flush=True)


if __name__ == "__main__":
    main(sys.argv[1:])
