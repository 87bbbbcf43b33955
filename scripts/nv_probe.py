#!/usr/bin/env python3
"""NVFP4 fused path (qz_quantize_nvfp4: k_nv_absmax + k_nv_encode) vs generic qz_quantize timing on the reference's NVFP4 shapes:
Qwen3-30B-A3B experts (4 resident layers rotated over 48, as bench.py's MXFP4 leg) and the
Qwen3-4B dense linears as grouped launches.  HIP events on the launch stream; prints one JSON
line per case.  Usage: python scripts/nv_probe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402
from test_nvfp4_gpu import two_pass  # noqa: E402

B_PER_PARAM = 2 + 0.5 + 1 / 16


def ev_time(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        fn()
        e1.record(st)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e-3
        best = t if best is None else min(best, t)
    return best


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    a = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn")
    g = torch.Generator(device=dev).manual_seed(0)
    layers = [((torch.randn(128, 1536, 2048, device=dev, generator=g) * 0.02).to(torch.bfloat16),
               (torch.randn(128, 2048, 768, device=dev, generator=g) * 0.02).to(torch.bfloat16)) for _ in range(4)]
    outs = {}
    for li, (gu, dn) in enumerate(layers):
        for j, w in enumerate((gu[:, :768], gu[:, 768:], dn)):
            outs[(li, j)] = ops.alloc_outputs(tuple(w.shape), a, None, dev)

    def moe(single):
        for li in range(48):
            gu, dn = layers[li % 4]
            for j, w in enumerate((gu[:, :768], gu[:, 768:], dn)):
                if single:
                    ops.quantize_weight(w, a, out=outs[(li % 4, j)])
                else:
                    two_pass(w, a)
    npar = 48 * 128 * 3 * 768 * 2048
    for name, single in (("fused", True), ("two_pass", False)):
        t = ev_time(lambda: moe(single))
        gbps = npar * B_PER_PARAM / t / 1e9
        print(json.dumps({"case": f"qwen3_30b_a3b_experts_nvfp4_{name}", "ms": t * 1e3, "params_per_s": npar / t,
                          "alg_GBps": gbps, "frac": gbps / 8000}), flush=True)
    # one fused-expert launch alone (the rocprof unit): gate half of layer 0
    w = layers[0][0][:, :768]
    o = outs[(0, 0)]
    t = ev_time(lambda: [ops.quantize_weight(w, a, out=o) for _ in range(20)]) / 20
    nb = w.numel() * B_PER_PARAM
    print(json.dumps({"case": "one_launch_128x768x2048", "us": t * 1e6, "frac": nb / t / 1e9 / 8000}), flush=True)
    del layers, outs
    torch.cuda.empty_cache()
    # dense Qwen3-4B NVFP4 (recipe_Dense_NVFP4): 36 layers x 7 linears, grouped per shape
    shapes = [(4096, 2560), (1024, 2560), (1024, 2560), (2560, 4096), (9728, 2560), (9728, 2560), (2560, 9728)]
    by = {}
    for l in range(36):
        for r, c in shapes:
            by.setdefault((r, c), []).append((torch.randn(r, c, device=dev, generator=g) * 0.02).to(torch.bfloat16))
    gqs = [ops.GroupedQuantize(ws, a) for ws in by.values()]
    npar = sum(w.numel() for ws in by.values() for w in ws)
    t = ev_time(lambda: [q.run() for q in gqs])
    gbps = npar * B_PER_PARAM / t / 1e9
    print(json.dumps({"case": "qwen3_4b_dense_nvfp4_grouped", "ms": t * 1e3, "params_per_s": npar / t,
                      "alg_GBps": gbps, "frac": gbps / 8000}), flush=True)
    for (r, c), q in zip(by.keys(), gqs):
        tq = ev_time(lambda: q.run())
        nb = q.n * r * c * B_PER_PARAM
        print(json.dumps({"case": f"grouped_{r}x{c}x{q.n}", "us": tq * 1e6, "frac": nb / tq / 1e9 / 8000}), flush=True)


if __name__ == "__main__":
    main()
