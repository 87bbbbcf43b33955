#!/usr/bin/env python3
"""Step-by-step comparison of transformers' fused-experts loop and awq._RoutedExpertsReplay on
the routing a Qwen3-30B-A3B-shaped router produces (random-init model, 4 layers, the CLI's
synthetic calibration tokens through layer 0): the first expert and op where they part.

  python scripts/moe_replay_probe2.py"""
import json
import os
import sys

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from transformers import AutoConfig, AutoModelForCausalLM
    from quantizers_amd.awq import _RoutedExpertsReplay
    dev = torch.device("cuda", 0)
    cfg = AutoConfig.from_pretrained(os.path.join(ROOT, "configs", "models", "qwen3-30b-a3b-4layers"))
    cfg.num_hidden_layers = 1
    torch.manual_seed(0)
    with torch.device(dev):
        m = AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)
    blk = m.model.layers[0].mlp
    ex = blk.experts
    g = torch.Generator().manual_seed(42)
    ids = torch.randint(0, cfg.vocab_size, (16, 2048), generator=g).to(dev)
    cap = {}
    h = blk.register_forward_pre_hook(lambda mod, a: cap.setdefault("x", a[0].detach().clone()))
    with torch.no_grad():
        m(ids[:1])  # one sample is enough to get realistic hidden states
    h.remove()
    x = cap["x"].reshape(-1, cfg.hidden_size)
    x = x.repeat(16, 1)
    with torch.no_grad():
        _, w, idx = blk.gate(x)
        counts = torch.bincount(idx.reshape(-1), minlength=cfg.num_experts)
        mask = nn.functional.one_hot(idx, num_classes=ex.num_experts).permute(2, 1, 0)
        hit = torch.greater(mask.sum(dim=(-1, -2)), 0).nonzero()
        fa = torch.zeros_like(x)
        fb = torch.zeros_like(x)
        first = None
        for eh in hit:
            eh = eh[0]
            e = int(eh)
            pos, tok = torch.where(mask[eh])
            ca = x[tok]
            ga, ua = nn.functional.linear(ca, ex.gate_up_proj[eh]).chunk(2, dim=-1)
            gb, ub = nn.functional.linear(ca, ex.gate_up_proj[e]).chunk(2, dim=-1)
            ha = ex.act_fn(ga) * ua
            hb = ex.act_fn(gb) * ub
            da = nn.functional.linear(ha, ex.down_proj[eh])
            db = nn.functional.linear(hb, ex.down_proj[e])
            da = da * w[tok, pos, None]
            db = db * w[tok, pos, None]
            fa.index_add_(0, tok, da.to(fa.dtype))
            fb.index_add_(0, tok, db.to(fb.dtype))
            if first is None:
                for name, a, b in (("gate_up", ga, gb), ("act*up", ha, hb), ("down*w", da, db), ("final", fa, fb)):
                    if not torch.equal(a, b):
                        first = {"expert": e, "tokens": int(tok.numel()), "op": name, "n_diff": int((a != b).sum())}
                        break
        ref = ex(x, idx, w)
        rp = _RoutedExpertsReplay(ex)
        got = rp._replay(x, w, rp._plan(idx))
    print(json.dumps({"tokens": int(x.shape[0]), "experts_hit": int(hit.numel()),
                      "tokens_per_expert_min_max": [int(counts.min()), int(counts.max())],
                      "w_dtype": str(w.dtype), "idx_dtype": str(idx.dtype),
                      "hf_loop_restated_equals_module": torch.equal(fa, ref),
                      "replay_equals_module": torch.equal(got, ref), "first_divergence": first}), flush=True)


if __name__ == "__main__":
    main()
