"""Clock-ramp probe: per-step HIP-event times from a cold start (0.5 s idle) for the bench
headline step (CompressionPlan, Qwen3-4B int4 g128), for library variants given as arguments
(ctypes, the plan's own tables), and for a plain torch copy moving the same bytes -- to tell a
platform ramp from a kernel-specific one.
usage: python scripts/ramp_probe.py [lib.so ...]"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from quantizers_amd import _lib  # noqa: E402
from quantizers_amd.compressor import CompressionPlan, compression_units  # noqa: E402

P, I64 = ctypes.c_void_p, ctypes.c_int64


def ramp(step, n=60):
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    time.sleep(0.5)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    ev[0].record(st)
    for i in range(n):
        step()
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(n)]


def show(name, us):
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    print(f"{name:22s} 0-9: " + " ".join(f"{u:5.0f}" for u in us[:10]) +
          f" | 5-24 mean {sum(us[5:25]) / 20:6.0f}  25-59 median {med(us[25:]):6.0f}", flush=True)


def main(paths):
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    model = bench.build_model(dev)
    plan = CompressionPlan(compression_units(model)[0], dev)
    sp = P(torch.cuda.current_stream().cuda_stream)
    calls = [(gq.n, P(gq.table.data_ptr()), gq.rows, gq.cols, gq.ca, gq.out_fmt) for gq, *_ in plan.grouped]
    libs = []
    for p in paths:
        lib = ctypes.CDLL(p)
        lib.qz_quantize_grouped.argtypes = [I64, P, I64, I64, ctypes.POINTER(_lib.QzArgs), ctypes.c_int32, P]
        libs.append((os.path.basename(p), lib))
    nbytes = plan.alg_bytes()
    src = torch.empty(nbytes // 2 // 2, dtype=torch.bfloat16, device=dev)
    dst = torch.empty_like(src)
    for rep in range(3):
        show("plan (in-tree lib)", ramp(lambda: plan.run()))
        for name, lib in libs:
            show(name, ramp(lambda lib=lib: [lib.qz_quantize_grouped(n, t, r, c, ctypes.byref(ca), f, sp)
                                             for n, t, r, c, ca, f in calls]))
        show("torch copy, same bytes", ramp(lambda: dst.copy_(src)))


if __name__ == "__main__":
    main(sys.argv[1:])
