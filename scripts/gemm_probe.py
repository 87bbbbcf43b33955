#!/usr/bin/env python3
"""hipBLASLt rate of the AWQ expert-search GEMM in its possible layouts (one expert, one grid
point: out[T, H] = h[T, I] @ Wq[H, I]^T), HIP-event timed over 50 launches after warmup.

  python scripts/gemm_probe.py"""
import json

import torch
import torch.nn.functional as F

SHAPES = {"qwen3_30b_a3b_w2": (32768, 768, 2048), "minimax_m2_1_w2": (16384, 1536, 3072)}


def timeit(fn, n=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    res = {}
    for name, (t, i, h) in SHAPES.items():
        x = torch.randn(t, i, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(h, i, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        wt = w.t().contiguous()
        xt = x.t().contiguous()
        flops = 2.0 * t * i * h
        ref = F.linear(x, w)
        variants = {
            "linear(x, w)": lambda: F.linear(x, w),
            "mm(x, wT contiguous)": lambda: torch.mm(x, wt),
            "mm(w, xT contiguous) -> [H, T]": lambda: torch.mm(w, xt),
            "mm(w, x.t())": lambda: torch.mm(w, x.t()),
        }
        row = {}
        for vn, fn in variants.items():
            us = timeit(fn)
            out = fn()
            same = torch.equal(out if out.shape == ref.shape else out.t(), ref)
            row[vn] = {"us": round(us, 1), "TFLOPs": round(flops / us / 1e6, 0), "bit_identical_to_linear": same}
        res[name] = row
        print(json.dumps({name: row}), flush=True)


if __name__ == "__main__":
    main()
