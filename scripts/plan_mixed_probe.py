#!/usr/bin/env python3
"""Whole Qwen3-4B int4-g128 (252 linears): the plan's 5 per-shape grouped launches vs ONE
mixed-shape grouped launch (qz_quantize_grouped_var), alternating, HIP events, best of 5 x 20
steps.  Usage: python scripts/plan_mixed_probe.py"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.compressor import compression_units  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = bench.build_model(dev)
    units, _ = compression_units(model)
    a = units[0].scheme.weights
    ws = [u.refs[0].weight for u in units]
    by = {}
    for w in ws:
        by.setdefault(tuple(w.shape), []).append(w)
    per_shape = [ops.GroupedQuantize(v, a) for v in by.values()]
    mixed = ops.GroupedQuantize([w for v in by.values() for w in v], a)
    assert mixed.mixed
    st = torch.cuda.current_stream()
    for rnd in range(3):
        for name, fn in (("per_shape", lambda: [g.run() for g in per_shape]), ("mixed", mixed.run)):
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            best = None
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(20):
                    fn()
                e1.record(st)
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / 20
                best = t if best is None else min(best, t)
            print(json.dumps({"round": rnd, "plan": name, "ms_per_step": best}), flush=True)


if __name__ == "__main__":
    main()
