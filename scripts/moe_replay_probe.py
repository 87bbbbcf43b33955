#!/usr/bin/env python3
"""Qwen3-30B-A3B-shaped fused experts (128 x [1536, 2048] gate_up, [2048, 768] down), 32,768
tokens with random top-8 routing: is the module's own forward deterministic run to run, and where
does the sync-free replay (awq._RoutedExpertsReplay) first differ from it?

  python scripts/moe_replay_probe.py"""
import json
import os
import sys

import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from transformers import AutoConfig
    from transformers.models.qwen3_moe.modeling_qwen3_moe import Qwen3MoeExperts
    from quantizers_amd.awq import _RoutedExpertsReplay
    dev = torch.device("cuda", 0)
    cfg = AutoConfig.from_pretrained(os.path.join(ROOT, "configs", "models", "qwen3-30b-a3b"))
    torch.manual_seed(0)
    with torch.device(dev):
        ex = Qwen3MoeExperts(cfg).to(torch.bfloat16)
        nn.init.normal_(ex.gate_up_proj, std=0.02)
        nn.init.normal_(ex.down_proj, std=0.02)
    t = 32768
    x = torch.randn(t, cfg.hidden_size, device=dev).to(torch.bfloat16)
    logits = torch.randn(t, cfg.num_experts, device=dev)
    w, idx = torch.topk(logits.softmax(-1), cfg.num_experts_per_tok, dim=-1)
    w = (w / w.sum(-1, keepdim=True)).to(torch.bfloat16)
    with torch.no_grad():
        a = ex(x, idx, w)
        b = ex(x, idx, w)
        rp = _RoutedExpertsReplay(ex)
        plan = rp._plan(idx)
        c = rp._replay(x, w, plan)
        # per-step comparison for the first routed expert
        e, pos, tok = plan[0]
        cur = x[tok]
        g1 = nn.functional.linear(cur, ex.gate_up_proj[e])
        g2 = nn.functional.linear(cur, ex.gate_up_proj[torch.tensor(e, device=dev)])
        g3 = nn.functional.linear(cur, ex.gate_up_proj[e].clone())
    res = {"module_forward_deterministic": torch.equal(a, b), "replay_equals_module": torch.equal(a, c),
           "n_diff_replay": int((a != c).sum()), "n_diff_rerun": int((a != b).sum()),
           "gemm_view_vs_tensor_index": torch.equal(g1, g2), "gemm_view_vs_clone": torch.equal(g1, g3),
           "tokens_first_expert": int(tok.numel())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
