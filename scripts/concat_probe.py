#!/usr/bin/env python3
"""Are per-batch GEMMs bit-identical to one GEMM over the concatenated batches (hipBLASLt, the
AWQ per-expert input shapes)?  If so the per-expert hidden states can be computed in one launch
instead of one per calibration batch without changing a bit.

  python scripts/concat_probe.py"""
import json
import time

import torch
import torch.nn.functional as F

CASES = {"qwen3_30b_a3b_gate_up": (16, 2048, 2048, 1536), "minimax_m2_1_w1": (8, 2048, 3072, 1536),
         "qwen3_4b_like": (16, 2048, 2560, 9728)}


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    for name, (nb, s, h, n) in CASES.items():
        xs = [torch.randn(s, h, device=dev, generator=g).to(torch.bfloat16) for _ in range(nb)]
        w = (torch.randn(n, h, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        per = torch.cat([F.linear(x, w) for x in xs])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        one = F.linear(torch.cat(xs), w)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        diff = (per.float() - one.float()).abs()
        print(json.dumps({name: {"bit_identical": torch.equal(per, one), "n_diff": int((diff > 0).sum()),
                                 "max_abs_diff": float(diff.max()), "per_batch_ms": round((t1 - t0) * 1e3, 2),
                                 "concat_ms": round((t2 - t1) * 1e3, 2)}}), flush=True)


if __name__ == "__main__":
    main()
