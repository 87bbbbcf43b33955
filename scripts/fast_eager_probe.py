#!/usr/bin/env python3
"""Can transformers' EAGER fused-experts arithmetic (per routed expert: GEMMs, routing weight,
bf16 index_add_ in ascending expert order -- the reference's transformers-4.57 loop) be computed
with two grouped GEMMs and a k-step bf16 accumulation, bit for bit?  Qwen3-30B-A3B and
MiniMax-M2.1 expert shapes, routing from a random router over 32,768 / 16,384 tokens.

  python scripts/fast_eager_probe.py"""
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def fast_eager(m, x, idx, w):
    t, k = idx.shape
    flat = idx.reshape(-1)
    e_sorted, perm = torch.sort(flat, stable=True)
    offs = torch.bincount(flat, minlength=m.num_experts).cumsum(0).to(torch.int32)
    xg = x[perm // k]
    gate, up = F.grouped_mm(xg, m.gate_up_proj.transpose(-2, -1), offs=offs).chunk(2, dim=-1)
    h = m.act_fn(gate) * up
    d = F.grouped_mm(h, m.down_proj.transpose(-2, -1), offs=offs)
    d = d * w.reshape(-1)[perm][:, None]
    contrib = torch.empty_like(d)
    contrib[perm] = d
    contrib = contrib.view(t, k, -1)
    order = torch.argsort(idx, dim=-1)
    contrib = torch.gather(contrib, 1, order[:, :, None].expand(-1, -1, contrib.shape[-1]))
    final = torch.zeros_like(x)
    for j in range(k):
        final = final + contrib[:, j]
    return final


def main():
    from transformers import AutoConfig
    from transformers.models.qwen3_moe.modeling_qwen3_moe import Qwen3MoeExperts
    dev = torch.device("cuda", 0)
    res = {}
    for name, cfgdir, tokens in (("qwen3_30b_a3b", "qwen3-30b-a3b", 32768), ("minimax_m2_1", "minimax-m2.1-2layers", 16384)):
        cfg = AutoConfig.from_pretrained(os.path.join(ROOT, "configs", "models", cfgdir))
        ne = getattr(cfg, "num_experts", None) or cfg.num_local_experts
        inter = getattr(cfg, "moe_intermediate_size", None) or cfg.intermediate_size
        cfg.num_experts, cfg.moe_intermediate_size = ne, inter
        cfg._experts_implementation = "eager"
        torch.manual_seed(0)
        with torch.device(dev):
            m = Qwen3MoeExperts(cfg).to(torch.bfloat16)
            torch.nn.init.normal_(m.gate_up_proj, std=0.02)
            torch.nn.init.normal_(m.down_proj, std=0.02)
        x = torch.randn(tokens, cfg.hidden_size, device=dev).to(torch.bfloat16)
        router = torch.randn(ne, cfg.hidden_size, device=dev).to(torch.bfloat16) * 0.02
        probs = F.linear(x, router).softmax(-1, dtype=torch.float)
        wv, idx = torch.topk(probs, cfg.num_experts_per_tok, dim=-1)
        wv = (wv / wv.sum(-1, keepdim=True)).to(torch.bfloat16)
        with torch.no_grad():
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ref = m(x, idx, wv)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            got = fast_eager(m, x, idx, wv)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            got = fast_eager(m, x, idx, wv)
            torch.cuda.synchronize()
            t3 = time.perf_counter()
            cfg._experts_implementation = "grouped_mm"
            m.config = cfg
            grp = m(x, idx, wv)
            torch.cuda.synchronize()
            t4 = time.perf_counter()
            grp = m(x, idx, wv)
            torch.cuda.synchronize()
            t5 = time.perf_counter()
        res[name] = {"fast_eager_bit_identical_to_eager": torch.equal(got.view(torch.int16), ref.view(torch.int16)),
                     "n_diff": int((got != ref).sum()), "grouped_mm_n_diff_vs_eager": int((grp != ref).sum()),
                     "ms_eager": round((t1 - t0) * 1e3, 1), "ms_fast_eager": round((t3 - t2) * 1e3, 1),
                     "ms_grouped_mm": round((t5 - t4) * 1e3, 1)}
        print(json.dumps({name: res[name]}), flush=True)


if __name__ == "__main__":
    main()
