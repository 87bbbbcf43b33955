"""Grouped quantize launch into output tensors never written before vs the same tensors again.
usage: python scripts/first_touch.py  (env: K=200)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402

ROWS, COLS = 11008, 4096
ALG = ROWS * COLS * 2 + ROWS * COLS // 2 + ROWS * COLS // 128 * 2


def timed(fn):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def main():
    K = int(os.environ.get("K", 200))
    dev = torch.device("cuda:0")
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    copies = [(torch.randn(ROWS, COLS, device=dev) * 0.02).to(torch.bfloat16) for _ in range(12)]
    ops.GroupedQuantize(copies[:2], a).run()
    torch.cuda.synchronize()
    for trial in range(3):
        torch.cuda.empty_cache()
        gq = ops.GroupedQuantize([copies[i % 12] for i in range(K)], a)  # fresh outputs
        res = [timed(gq.run) for _ in range(4)]
        zero = [{k: (torch.zeros_like(v) if v is not None else None) for k, v in o.items()} for o in gq.outs]
        torch.cuda.synchronize()
        gz = ops.GroupedQuantize([copies[i % 12] for i in range(K)], a, outs=zero)  # outputs pre-written by memset
        rz = [timed(gz.run) for _ in range(2)]
        print(f"trial {trial}: fresh outputs, launches 1..4: " +
              " ".join(f"{x * 1e3 / K:.2f}" for x in res) + " us/weight; memset-touched outputs: " +
              " ".join(f"{x * 1e3 / K:.2f}" for x in rz) + " us/weight", flush=True)
        del gq, gz, zero


if __name__ == "__main__":
    main()
