#!/usr/bin/env python3
"""Generate tests/golden/awq_int4_g128.safetensors from the CPU oracle
(oracle/ct_torch.py): one AWQ mapping whose parent is its single balance linear (the up -> down
shape of a Qwen3 MLP, K = 2560), int4 symmetric group 128.

  inputs   x [64, 2560] bf16 (per-channel magnitudes spread over 3 decades), w [128, 2560] bf16
  outputs  x_mean f32 [2560]          mean |x| over tokens (f32 sums, D8)
           w_mean f64 [2560]          mean over rows of |w| / bf16(group absmax + 1e-6)
           scales f32 [20, 2560]      the 20 grid points' scale vectors (duo scaling, fp32)
           losses f64 [20]            mean((bf16(x @ w^T) - bf16(x @ Q(w*s)/s^T))^2)
           best   i64 [1]             first argmin of the losses
           fq_best bf16 [128, 2560]   Q(w*s_best)/s_best
           smoothed bf16 [128, 2560]  bf16(w * s_best) (the applied smoothing of the balance layer)

The parent forward is torch's CPU bf16 linear: the GPU tests compare their own device forward to
the losses with a tolerance (GEMM summation order), everything else bit for bit.

``awq_int4_g128_bf16.safetensors`` (round 5, ``build(literal=True)``): the same mapping under
D8's bf16 reading (ct_torch.*_literal: x_mean / w_mean / scales bf16, W * s and the smoothing
with bf16 scales; the loss stays an f64 sum as the product computes it)."""
import os
import sys

import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "oracle"))
import ct_torch as ct  # noqa: E402

OUT = os.path.join(HERE, "awq_int4_g128.safetensors")
OUT_BF16 = os.path.join(HERE, "awq_int4_g128_bf16.safetensors")


def build(literal: bool = False):
    g = torch.Generator().manual_seed(2025)
    K, N, T = 2560, 128, 64
    mag = 10.0 ** (torch.rand(K, generator=g) * 3 - 2)  # channel magnitudes 0.01 .. 10
    x = (torch.randn(T, K, generator=g) * mag).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g) * 0.02).to(torch.bfloat16)
    a = ct.QArgs(num_bits=4, type="int", symmetric=True, group_size=128)
    if literal:
        x_mean, _ = ct.awq_accumulate_mean_literal(x)
        w_mean = ct.awq_layer_means_literal([w], a)
    else:
        s_sum, n = ct.awq_accumulate_mean(x)
        x_mean = s_sum / n
        w_mean = ct.awq_layer_means([w], a)
    ref = torch.nn.functional.linear(x, w)
    scales, losses, fqs = [], [], []
    for i in range(20):
        if literal:
            s = ct.awq_grid_scales_literal(x_mean, w_mean, i / 20, True)
            fq = ct.awq_fake_quant_scaled_literal(w, s, a)
        else:
            s = ct.awq_grid_scales(x_mean, w_mean.float(), i / 20, True)
            fq = ct.awq_fake_quant_scaled(w, s, a)
        out = torch.nn.functional.linear(x, fq)
        losses.append((ref - out).double().pow(2).sum().item() / ref.numel())
        scales.append(s)
        fqs.append(fq)
    best = min(range(20), key=lambda i: (losses[i], i))
    if literal:  # bf16 statistics and scales as they are
        return {"x": x, "w": w, "x_mean": x_mean, "w_mean": w_mean, "scales": torch.stack(scales),
                "losses": torch.tensor(losses, dtype=torch.float64), "best": torch.tensor([best], dtype=torch.int64),
                "fq_best": fqs[best], "smoothed": w * scales[best].view(1, -1)}
    return {
        "x": x, "w": w, "x_mean": x_mean.float(), "w_mean": w_mean.double(), "scales": torch.stack(scales),
        "losses": torch.tensor(losses, dtype=torch.float64), "best": torch.tensor([best], dtype=torch.int64),
        "fq_best": fqs[best], "smoothed": (w.float() * scales[best].view(1, -1)).to(torch.bfloat16),
    }


if __name__ == "__main__":
    for lit, out in ((False, OUT), (True, OUT_BF16)):
        t = build(lit)
        save_file({k: v.contiguous() for k, v in t.items()}, out)
        print(out, "best", int(t["best"]), [round(v, 9) for v in t["losses"].tolist()])
