"""Interleaved A/B of two CompressionPlan builds over the same model (the bench headline's
Qwen3-4B int4 g128, or RECIPE=mixed): row-block merged launches (compressor.ROW_BLOCKS) vs one
launch per shape.  Every on-disk tensor is compared bit for bit between the two; HIP events
around K back-to-back steps, median of ROUNDS.
usage: python scripts/plan_ab.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from quantizers_amd import compressor  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(7)
    recipe = bench.MIXED_RECIPE if os.environ.get("RECIPE") == "mixed" else bench.RECIPE
    model = bench.build_model(dev, recipe)
    units = compressor.compression_units(model)[0]
    plans = {}
    for name, rb in (("per_shape", False), ("row_blocks", True)):
        compressor.ROW_BLOCKS = rb
        plans[name] = compressor.CompressionPlan(units, dev)
        print(f"{name}: {plans[name].launches} launches", flush=True)
    outs = {}
    for name, p in plans.items():
        p.run()
        torch.cuda.synchronize()
        outs[name] = {k: v.clone() for k, v in p.tensors().items()}
    a, b = outs["per_shape"], outs["row_blocks"]
    same = a.keys() == b.keys() and all(torch.equal(a[k].view(-1).view(torch.uint8) if a[k].is_cuda else a[k],
                                                    b[k].view(-1).view(torch.uint8) if b[k].is_cuda else b[k])
                                        for k in a)
    print(f"bit-identical: {same}", flush=True)
    del outs, a, b
    k, rounds = int(os.environ.get("K", 20)), int(os.environ.get("ROUNDS", 15))
    res = {n: [] for n in plans}
    st = torch.cuda.current_stream()
    for _ in range(rounds):
        for n, p in plans.items():
            for _ in range(3):
                p.run(st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(k):
                p.run(st)
            e1.record(st)
            torch.cuda.synchronize()
            res[n].append(e0.elapsed_time(e1) * 1e3 / k)
    for n, v in res.items():
        v = sorted(v)
        print(f"{n:11s} step median {v[len(v) // 2]:8.2f} us  min {v[0]:8.2f} us  "
              f"frac {plans[n].alg_bytes() / (v[len(v) // 2] * 1e-6) / 8e12:.4f}", flush=True)


if __name__ == "__main__":
    main()
