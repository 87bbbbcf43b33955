#!/usr/bin/env python3
"""Does a second read of an NVFP4 batch come from the 256 MiB Infinity Cache (MALL)?  Per batch size,
qz_quantize_nvfp4 (two launches: |w| max, encode) on the SAME batch back to back (hot: after the
first call both reads can hit the MALL when the batch fits) vs rotating over 8 batches (cold).
Prints us per call and the algorithmic fraction of 8 TB/s.  Usage: python scripts/nv_mall_probe.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402


def ev(fn, n=20):
    fn(0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    dev = torch.device("cuda:0")
    a = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn")
    g = torch.Generator(device=dev).manual_seed(0)
    for slices in (8, 16, 32, 64, 128):
        ws = [(torch.randn(slices, 768, 2048, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(8)]
        out = ops.alloc_outputs(tuple(ws[0].shape), a, None, dev)
        nb = ws[0].numel() * (2 + 0.5 + 1 / 16)
        hot = ev(lambda i: ops.quantize_weight(ws[0], a, out=out))
        cold = ev(lambda i: ops.quantize_weight(ws[i % 8], a, out=out))
        print(json.dumps({"MB": ws[0].numel() * 2 / 1e6, "hot_us": hot, "cold_us": cold,
                          "hot_frac": nb / hot / 1e6 / 8, "cold_frac": nb / cold / 1e6 / 8}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def chunked():
    """The [128, 768, 2048] batch (403 MB) as consecutive sub-batch calls of 4 .. 128 slices."""
    dev = torch.device("cuda:0")
    a = QuantizationArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn")
    g = torch.Generator(device=dev).manual_seed(1)
    ws = [(torch.randn(128, 768, 2048, device=dev, generator=g) * 0.02).to(torch.bfloat16) for _ in range(3)]
    out = ops.alloc_outputs((128, 768, 2048), a, None, dev)
    nb = ws[0].numel() * (2 + 0.5 + 1 / 16)
    for c in (4, 8, 16, 32, 64, 128):
        def run(i, c=c):
            w = ws[i % 3]
            for s0 in range(0, 128, c):
                o = {k: v[s0:s0 + c] for k, v in out.items() if v is not None}
                ops.quantize_weight(w[s0:s0 + c], a, out=o)
        t = ev(run, 10)
        print(json.dumps({"chunk_slices": c, "chunk_MB": c * 768 * 2048 * 2 / 1e6, "us_per_403MB": t,
                          "frac": nb / t / 1e6 / 8}), flush=True)


if __name__ == "__main__" and len(sys.argv) > 1:
    chunked()
