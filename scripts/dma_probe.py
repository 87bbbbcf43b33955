#!/usr/bin/env python3
"""Host -> device DMA rate by the state of the DESTINATION device memory: the 252 Qwen3-4B
linear weights (7.27 GB, host, filled) copied through ``H2DStager`` into
  fresh      -- tensors allocated after ``empty_cache`` (new hipMalloc segments)
  reused_k   -- the caching allocator's blocks last written by a compute kernel (fill_)
  reused_dma -- the same destination tensors a second time (last written by the DMA engine)
  prefilled  -- destinations allocated, filled by a kernel, then copied into (copy_, no alloc)

  python scripts/dma_probe.py"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd.staging import H2DStager  # noqa: E402

SHAPES = [(4096, 2560), (1024, 2560), (1024, 2560), (2560, 4096), (9728, 2560), (9728, 2560), (2560, 9728)]


def timed(fn, st):
    torch.cuda.synchronize()
    for k in st.stats:
        st.stats[k] = 0 if k == "bytes" else 0.0
    t0 = time.perf_counter()
    out = fn()
    st.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return out, {"s": round(dt, 3), "GBps": round(st.stats["bytes"] / dt / 1e9, 1), "wait_s": round(st.stats["wait_s"], 3)}


def main():
    dev = torch.device("cuda", 0)
    ws = [torch.empty(s, dtype=torch.bfloat16).fill_(0.25) for _ in range(36) for s in SHAPES]
    st = H2DStager(dev)
    torch.empty(1, device=dev)
    res = {}
    for rnd in range(2):
        torch.cuda.empty_cache()
        _, res[f"fresh_{rnd}"] = timed(lambda: [st.copy(w) for w in ws], st)
        torch.cuda.empty_cache()
        # blocks written by a kernel, freed, then handed out again by the caching allocator
        tmp = [torch.empty(w.shape, dtype=w.dtype, device=dev).fill_(1.0) for w in ws]
        torch.cuda.synchronize()
        del tmp
        outs, res[f"reused_k_{rnd}"] = timed(lambda: [st.copy(w) for w in ws], st)
        del outs
        outs, res[f"reused_dma_{rnd}"] = timed(lambda: [st.copy(w) for w in ws], st)
        del outs
        pre = [torch.empty(w.shape, dtype=w.dtype, device=dev).fill_(1.0) for w in ws]
        torch.cuda.synchronize()

        def into():
            with torch.cuda.stream(st.stream):
                for d, w in zip(pre, ws):
                    d.copy_(w, non_blocking=False)
            st.stats["bytes"] = sum(w.numel() * 2 for w in ws)
            return None
        _, res[f"prefilled_pageable_copy_{rnd}"] = timed(into, st)
        del pre
        print(json.dumps({k: v for k, v in res.items() if k.endswith(str(rnd))}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
