#!/usr/bin/env python3
"""Run each north-star kernel a fixed number of times on the [11008, 4096] bf16 headline weight
(12 rotating HBM-resident copies, > the 256 MiB Infinity Cache) -- the program the rocprofv3
PMC passes of scripts/pmc_kernels.sh profile.  Prints per-kernel HIP-event times.

  python scripts/kernel_driver.py [N]      (N launches per kernel, default 30)
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402

R, C, G = 11008, 4096, 128


def main(n=30):
    dev = torch.device("cuda:0")
    gen = torch.Generator(device=dev).manual_seed(0)
    copies = [(torch.randn(R, C, device=dev, generator=gen) * 0.02).to(torch.bfloat16) for _ in range(12)]
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=G)
    s = torch.rand(C, device=dev, generator=gen) + 0.5
    fq_out = [torch.empty_like(copies[0]) for _ in range(4)]
    x = [torch.randn(16384, C, device=dev, generator=gen).to(torch.bfloat16) for _ in range(4)]
    sums = torch.zeros(C, dtype=torch.float32, device=dev)
    wsum = torch.zeros(C, dtype=torch.float64, device=dev)
    outs = [ops.alloc_outputs((R, C), a, None, dev) for _ in range(n)]
    prep = ops.PreparedQuantize(copies[0], a, outs[0])
    many = prep.prepare_many([copies[i % 12] for i in range(n)], outs=outs)
    gq = ops.GroupedQuantize([copies[i % 12] for i in range(n)], a, outs=outs)
    kernels = [
        ("quantize_per_weight", lambda i: prep.run(copies[i % 12]), 1),
        ("fake_quant_cols", lambda i: ops.fake_quantize(copies[i % 12], a, col_scales=s, out=fq_out[i % 4]), 1),
        ("absmean", lambda i: ops.awq_absmean_accum(x[i % 4], sums), 1),
        ("weight_mean", lambda i: ops.awq_weight_mean_accum(copies[i % 12], G, wsum), 1),
        ("scale_columns", lambda i: ops.scale_columns_(copies[i % 12], s), 1),
    ]
    st = torch.cuda.current_stream()
    for name, fn, _ in kernels:
        for i in range(3):
            fn(i)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for i in range(n):
            fn(i)
        e1.record(st)
        torch.cuda.synchronize()
        print(f"{name:22s} {e0.elapsed_time(e1) * 1e3 / n:8.2f} us/launch (events over {n} launches)", flush=True)
    many()
    gq.run()
    torch.cuda.synchronize()
    time.sleep(0.01)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
