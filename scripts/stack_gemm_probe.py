#!/usr/bin/env python3
"""Expert-search GEMMs: one torch.mm per grid point ([T, I] x [I, H], the current path) vs the
grid points stacked along N (one [T, I] x [I, G*H] GEMM), Qwen3-30B-A3B w2 shape (T = 32,768
calibration tokens, I = 768, H = 2048).  Prints HIP-event times and whether the stacked output
is bit-identical to the per-point outputs.  Usage: python scripts/stack_gemm_probe.py"""
import json

import torch


def ev(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e-3
        best = t if best is None else min(best, t)
    return best


def main():
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(0)
    T, I, H = 32768, 768, 2048
    h = (torch.randn(T, I, device=dev, generator=g) * 0.5).to(torch.bfloat16)
    for G in (4, 8):
        w = (torch.randn(G, H, I, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        outs = [torch.empty(T, H, dtype=torch.bfloat16, device=dev) for _ in range(G)]
        big = torch.empty(T, G * H, dtype=torch.bfloat16, device=dev)
        wt = w.reshape(G * H, I)

        def per_point():
            for k in range(G):
                torch.mm(h, w[k].t(), out=outs[k])

        def stacked():
            torch.mm(h, wt.t(), out=big)
        t1, t2 = ev(per_point), ev(stacked)
        same = all(torch.equal(outs[k], big[:, k * H:(k + 1) * H]) for k in range(G))
        fl = 2 * T * I * H * G
        print(json.dumps({"grid_points": G, "per_point_us": t1 * 1e6 / G, "stacked_us_per_point": t2 * 1e6 / G,
                          "per_point_TFLOPs": fl / t1 / 1e12, "stacked_TFLOPs": fl / t2 / 1e12,
                          "bit_identical": same}), flush=True)


if __name__ == "__main__":
    main()
