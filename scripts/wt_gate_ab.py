"""Interleaved A/B of whole-library builds on the three int4-g128 launch patterns the write-through
tail touches, in the bench's own cold pattern:

  per_weight  100 one-weight [11008, 4096] launches (qz_quantize_many) over 12 rotating HBM-resident
              copies into 100 distinct output sets (bench.py synthetic_leg "per_weight")
  grouped     ONE grouped launch over the same 100 weights / outputs (synthetic_leg "grouped")
  plan        K whole headline steps: CompressionPlan over Qwen3-4B (5 grouped launches per step)

Every round runs each library's three legs in turn; outputs are bit-checked against the first
library.  HIP-event medians are printed here; under rocprofv3 --kernel-trace the launch order is
written to SEQ (one line per block: lib leg launches), so scripts/wt_gate_rocprof.py can attribute
every kernel record to its library and leg and take rocprof medians.

usage: SEQ=gpurun_out/x.seq python scripts/wt_gate_ab.py lib_a.so lib_b.so ...
"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from quantizers_amd import _lib, ops  # noqa: E402
from quantizers_amd.compressor import CompressionPlan, compression_units  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402

P = ctypes.c_void_p
R, C, G = 11008, 4096, 128


def main(paths):
    ref = _lib.load()
    libs = []
    for p in paths:
        lib = ctypes.CDLL(p)
        for fn in ("qz_quantize_many", "qz_quantize_grouped"):
            getattr(lib, fn).argtypes = getattr(ref, fn).argtypes
            getattr(lib, fn).restype = getattr(ref, fn).restype
        libs.append(lib)
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(99)
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, strategy="group", group_size=G)
    ca = a.to_c()
    copies = [(torch.randn(R, C, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for _ in range(12)]
    k = 100
    ws = [copies[i % 12] for i in range(k)]
    outs = [ops.alloc_outputs((R, C), a, None, dev) for _ in range(k)]
    gq = ops.GroupedQuantize(ws, a, outs=outs)
    wsp = torch.empty(max(256, ref.qz_quantize_workspace_size(1, R, C, ctypes.byref(ca))), dtype=torch.uint8, device=dev)
    arr = lambda ts: (P * k)(*[t.data_ptr() for t in ts])  # noqa: E731
    w_arr, q_arr, s_arr = arr(ws), arr([o["codes"] for o in outs]), arr([o["scale"] for o in outs])
    torch.manual_seed(7)
    model = bench.build_model(dev)
    plan = CompressionPlan(compression_units(model)[0], dev)
    calls = [(g.n, P(g.table.data_ptr()), g.rows, g.cols, g.ca, g.out_fmt) for g, *_ in plan.grouped]
    st = torch.cuda.current_stream()
    sp = P(st.cuda_stream)
    seq_path = os.environ.get("SEQ")
    seq = open(seq_path, "w") if seq_path else None
    steps = int(os.environ.get("K", 10))

    # one-entry grouped tables (register loads, GRP kernel) per weight, into the same 100 outputs
    tabs = [torch.tensor([[ws[i].data_ptr()], [outs[i]["codes"].data_ptr()], [outs[i]["scale"].data_ptr()], [0]],
                         dtype=torch.int64).reshape(-1).to(dev) for i in range(k)]
    tab_ptrs = [P(t.data_ptr()) for t in tabs]
    one = [P(outs[0]["codes"].data_ptr())] * k, [P(outs[0]["scale"].data_ptr())] * k
    q1_arr, s1_arr = (P * k)(*one[0]), (P * k)(*one[1])

    def leg(lib, name, reps=1):
        if name == "pw_grp":  # one-weight launches of the grouped (register-load) kernel
            for _ in range(reps):
                for tp in tab_ptrs:
                    rc = lib.qz_quantize_grouped(1, tp, R, C, ctypes.byref(gq.ca), gq.out_fmt, sp)
                    assert rc == 0, rc
            return k * reps
        if name == "pw_same":  # scripts/kernel_driver.py's pattern: every launch into ONE output set
            for _ in range(reps):
                rc = lib.qz_quantize_many(k, w_arr, q1_arr, s1_arr, None, None, 1, R, C, C, R * C, ctypes.byref(ca),
                                          _lib.QZ_OUT_PACKED_INT32, P(wsp.data_ptr()), wsp.numel(), sp)
                assert rc == 0, rc
            return k * reps
        if name == "per_weight":
            for _ in range(reps):
                rc = lib.qz_quantize_many(k, w_arr, q_arr, s_arr, None, None, 1, R, C, C, R * C, ctypes.byref(ca),
                                          _lib.QZ_OUT_PACKED_INT32, P(wsp.data_ptr()), wsp.numel(), sp)
                assert rc == 0, rc
            return k * reps
        if name == "grouped":
            for _ in range(reps):
                rc = lib.qz_quantize_grouped(k, P(gq.table.data_ptr()), R, C, ctypes.byref(gq.ca), gq.out_fmt, sp)
                assert rc == 0, rc
            return reps
        for _ in range(reps):
            for n, tab, r, c, cc, fmt in calls:
                rc = lib.qz_quantize_grouped(n, tab, r, c, ctypes.byref(cc), fmt, sp)
                assert rc == 0, rc
        return reps * len(calls)

    def snap():
        torch.cuda.synchronize()
        return ([torch.cat([o["codes"].reshape(-1).view(torch.uint8), o["scale"].reshape(-1).view(torch.uint8)])
                 for o in outs[::17]] +
                [torch.cat([o["codes"].reshape(-1).view(torch.uint8) for o in g.outs]) for g, *_ in plan.grouped])

    base = None
    for p, lib in zip(paths, libs):
        n = leg(lib, "per_weight") + leg(lib, "plan")
        if seq:
            seq.write(f"{os.path.basename(p)} check {n}\n")
        got = snap()
        if base is None:
            base = got
        else:
            print(f"{os.path.basename(p)}: outputs {'identical' if all(torch.equal(x, y) for x, y in zip(base, got)) else 'MISMATCH'}",
                  flush=True)
    rounds = int(os.environ.get("ROUNDS", 7))
    legs = os.environ.get("LEGS", "per_weight,pw_same,grouped,plan").split(",")
    res = {(p, l): [] for p in paths for l in legs}
    for _ in range(rounds):
        for p, lib in zip(paths, libs):
            for name, reps in [(l, {"grouped": 3, "plan": steps}.get(l, 1)) for l in legs]:
                n = leg(lib, name, 1 if name != "plan" else 2)  # warm: the same pattern once
                if seq:
                    seq.write(f"{os.path.basename(p)} warm {n}\n")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                n = leg(lib, name, reps)
                e1.record(st)
                torch.cuda.synchronize()
                if seq:
                    seq.write(f"{os.path.basename(p)} {name} {n}\n")
                per = {"per_weight": k, "pw_same": k, "pw_grp": k, "grouped": k * reps, "plan": reps}[name]
                res[(p, name)].append(e0.elapsed_time(e1) * 1e3 / per)
    for name, unit in (("per_weight", "us/launch"), ("pw_same", "us/launch"), ("pw_grp", "us/launch"),
                       ("grouped", "us/weight"), ("plan", "us/step")):
        if name not in legs:
            continue
        for p in paths:
            v = sorted(res[(p, name)])
            print(f"{name:11s} {os.path.basename(p):18s} event median {v[len(v) // 2]:9.2f} {unit}  min {v[0]:9.2f}",
                  flush=True)
    if seq:
        seq.close()


if __name__ == "__main__":
    main(sys.argv[1:])
