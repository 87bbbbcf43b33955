#!/usr/bin/env python3
"""Host -> device weight staging A/B: the 252 Qwen3-4B linear weights (7.27 GB bf16, host,
pageable) moved as one ``tensor.to(device)`` per weight (the pre-r02ab save path) vs through
``staging.H2DStager`` (two pinned 256 MB buffers, DMA on a side stream), interleaved, 3 rounds.
Every timed copy reads freshly allocated host tensors (a save path copies each weight once: the
pages have never been DMA'd) -- plus, as "warm", a second copy of the same tensors.

  python scripts/ab_stage.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd.staging import H2DStager  # noqa: E402

SHAPES = [(4096, 2560), (1024, 2560), (1024, 2560), (2560, 4096), (9728, 2560), (9728, 2560), (2560, 9728)]


def main():
    dev = torch.device("cuda", 0)

    def fresh():
        return [torch.empty(s, dtype=torch.bfloat16).fill_(0.5) for _ in range(36) for s in SHAPES]

    st = H2DStager(dev)
    torch.empty(1, device=dev).copy_(torch.ones(1))  # runtime initialised before any timing
    res = {"weights": 36 * len(SHAPES), "rounds": []}
    for r in range(3):
        row = {}
        order = ("to_per_weight", "stager") if r % 2 == 0 else ("stager", "to_per_weight")
        for name in order:
            ws = fresh()
            nb = sum(w.numel() * 2 for w in ws)
            res["bytes"] = nb
            for phase in ("cold", "warm"):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if name == "to_per_weight":
                    out = [w.to(dev) for w in ws]
                else:
                    out = [st.copy(w) for w in ws]
                    st.wait()
                torch.cuda.synchronize()
                dt = time.perf_counter() - t0
                assert torch.equal(out[-1][:2].cpu(), ws[-1][:2])
                del out
                torch.cuda.empty_cache()
                row[f"{name}_{phase}"] = {"s": round(dt, 4), "GBps": round(nb / dt / 1e9, 1)}
            del ws
        res["rounds"].append(row)
        print(json.dumps(row), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
