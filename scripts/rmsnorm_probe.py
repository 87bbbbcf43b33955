#!/usr/bin/env python3
"""Which summation tree and rsqrt reproduce PyTorch's Qwen3RMSNorm over 128-wide rows bit for bit?
Emulates the candidate trees with explicit f32 adds against torch's own mean, compares
torch.rsqrt with the correctly rounded f64 value, and checks qz_rmsnorm128 (built from the
answer) against the module's forward on random bf16 rows at several scales.
(profiles/r03t_rmsnorm_probe.log is the run that settled it, when the kernel still had the
candidates as variants: 64-lane trees, v_rsq_f32, rsqrtf and 1/sqrtf all differed.)
python scripts/rmsnorm_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from quantizers_amd import ops  # noqa: E402

from transformers.models.qwen3.modeling_qwen3 import Qwen3RMSNorm  # noqa: E402

dev = torch.device("cuda", 0)
norm = Qwen3RMSNorm(128, eps=1e-6).to(dev).to(torch.bfloat16)
g = torch.Generator(device=dev).manual_seed(0)
with torch.no_grad():
    norm.weight.copy_((torch.rand(128, generator=g, device=dev) * 2).to(torch.bfloat16))
    for scale in (1e-3, 1.0, 30.0):
        x = (torch.randn(65536, 8, 128, generator=g, device=dev) * scale).to(torch.bfloat16)
        want = norm(x)
        line = []
        got = ops.rmsnorm128(x, norm.weight, norm.variance_epsilon)
        bad = (got.view(torch.int16) != want.view(torch.int16)).sum().item()
        line.append(f"qz_rmsnorm128: {bad} of {want.numel()} differ")
        print(f"scale {scale}: " + "; ".join(line), flush=True)

    # which summation tree is torch's mean over 128?  emulate the candidates with explicit f32 adds
    def tree_down(v, increasing):  # v [..., n] lanes; shuffle-down tree, lane 0's value
        n = v.shape[-1]
        offs = [1 << i for i in range(n.bit_length() - 1)]
        for off in (offs if increasing else offs[::-1]):
            shifted = torch.cat([v[..., off:], v[..., n - off:]], dim=-1)  # out-of-range lanes keep their own
            v = v + shifted
        return v[..., 0]

    x = (torch.randn(262144, 128, generator=g, device=dev)).to(torch.bfloat16)
    sq = x.float().pow(2)
    ref = sq.mean(-1)
    leaves64 = sq[:, :64] + sq[:, 64:]
    leaves32 = ((sq[:, 0::4] + sq[:, 1::4]) + sq[:, 2::4]) + sq[:, 3::4]
    cands = {"64 lanes (t, t+64), offsets up": tree_down(leaves64, True),
             "64 lanes (t, t+64), offsets down": tree_down(leaves64, False),
             "32 lanes x4 vector, offsets up": tree_down(leaves32, True),
             "32 lanes x4 vector, offsets down": tree_down(leaves32, False),
             "sequential": sq.cumsum(-1)[:, -1],
             "pairwise halves": None}
    h = sq
    while h.shape[-1] > 1:
        h = h[:, : h.shape[-1] // 2] + h[:, h.shape[-1] // 2:]
    cands["pairwise halves"] = h[:, 0]
    for name, s in cands.items():
        print(f"mean tree {name}: {(s * (1.0 / 128) != ref).sum().item()} of {ref.numel()} rows differ", flush=True)
    y = ref + 1e-6
    r_t = torch.rsqrt(y)
    print("torch.rsqrt vs 1/sqrt (f32):", (r_t != 1.0 / torch.sqrt(y)).sum().item(),
          "vs f64 rounded once:", (r_t != (1.0 / y.double().sqrt()).float()).sum().item(), "of", y.numel(), flush=True)
    # the final steps: bf16(x * r) and bf16(w * y) against the module, with torch's own r
    xf = x.float()
    y1 = (xf * r_t[:, None]).to(torch.bfloat16)
    emu = norm.weight * y1
    print("module vs composed with torch.rsqrt:", (norm(x).view(torch.int16) != emu.view(torch.int16)).sum().item(),
          flush=True)
