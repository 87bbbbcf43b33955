"""Row-pitch probe of the AWQ statistics kernels: the same [rows, cols] operand read from buffers
of different row pitch (ld), so the plan (chunks, windows) is fixed and only the addresses move.
usage: python scripts/stride_probe.py   (HIP events over 50 calls, 8 rotating buffers each)"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402


def timed(fn, n=50):
    for i in range(5):
        fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(n):
        fn(i)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


def main():
    dev = torch.device("cuda:0")
    for which, rows, cols, lds in (("wmean", 19456, 2560, (2560, 2816, 3072, 4096, 5120)),
                                   ("wmean", 11008, 4096, (4096, 4352, 5120, 6144, 8192)),
                                   ("absmean", 32768, 2560, (2560, 3072, 4096)),
                                   ("absmean", 16384, 4096, (4096, 5120, 8192))):
        for ld in lds:
            bufs = [torch.randn(rows, ld, device=dev).to(torch.bfloat16) * 0.02 for _ in range(8)]
            views = [b[:, :cols] for b in bufs]
            if which == "wmean":
                out = torch.zeros(cols, dtype=torch.float64, device=dev)
                us = timed(lambda i: ops.awq_weight_mean_accum(views[i % 8], 128, out))
            else:
                out = torch.zeros(cols, dtype=torch.float32, device=dev)
                us = timed(lambda i: ops.awq_absmean_accum(views[i % 8], out))
            nb = rows * cols * 2
            print(f"{which:8s} [{rows}, {cols}] ld {ld:5d}: {us:7.2f} us  {nb / us / 1e6:6.3f} TB/s  "
                  f"frac {nb / us / 1e6 / 8:.3f}", flush=True)
            del bufs, views
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
