"""Does an idle gap before a grouped launch slow it down (clock ramp)?  Times one grouped launch
(K weights, distinct outputs) after: a host sleep of S ms following a sync, or directly behind
another launch on the stream.  usage: python scripts/idle_gap.py  (env: K=200)"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402
from quantizers_amd.quantization import QuantizationArgs  # noqa: E402

ROWS, COLS = 11008, 4096


def main():
    K = int(os.environ.get("K", 200))
    dev = torch.device("cuda:0")
    a = QuantizationArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    copies = [(torch.randn(ROWS, COLS, device=dev) * 0.02).to(torch.bfloat16) for _ in range(12)]
    gq = ops.GroupedQuantize([copies[i % 12] for i in range(K)], a)
    small = ops.GroupedQuantize([copies[i % 12] for i in range(20)], a)
    gq.run()
    torch.cuda.synchronize()
    res = {}
    for rnd in range(4):
        for gap in (0.0, 0.001, 0.01, 0.1, "behind", "behind_small"):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            if gap == "behind":
                gq.run()
            elif gap == "behind_small":
                small.run()
            else:
                time.sleep(gap)
            e0.record()
            gq.run()
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(gap, []).append(e0.elapsed_time(e1) * 1e3 / K)
    for gap, v in res.items():
        print(f"before the launch: {str(gap):12s} us/weight: " + " ".join(f"{x:.2f}" for x in v), flush=True)


if __name__ == "__main__":
    main()
