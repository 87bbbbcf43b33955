"""Per-step times of the bench headline (the whole-model CompressionPlan, Qwen3-4B int4 g128)
from a cold start: one event pair per step over W + K steps, printed in order, to show how many
steps the clocks need after the host-side set-up (bench.py times K = 20 steps after W = 5).
usage: python scripts/step_ramp.py [steps]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from quantizers_amd.compressor import CompressionPlan, compression_units  # noqa: E402


def main(n=200):
    dev = torch.device("cuda:0")
    torch.manual_seed(1234)
    model = bench.build_model(dev)
    plan = CompressionPlan(compression_units(model)[0], dev)
    st = torch.cuda.current_stream(dev)
    torch.cuda.synchronize()
    for gap in (0.0, 0.5):
        time.sleep(gap)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        ev[0].record(st)
        for i in range(n):
            plan.run(st)
            ev[i + 1].record(st)
        torch.cuda.synchronize()
        us = [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(n)]
        print(f"after {gap:.1f} s idle: steps 0-9 " + " ".join(f"{u:.0f}" for u in us[:10]), flush=True)
        for a, b in ((0, 5), (5, 25), (25, 50), (50, 100), (100, n)):
            seg = sorted(us[a:b])
            print(f"  steps {a:3d}-{b - 1:3d}: median {seg[len(seg) // 2]:7.1f} us  mean {sum(seg) / len(seg):7.1f} us",
                  flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
