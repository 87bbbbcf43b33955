"""CPU: checkpoint naming of fused MoE experts and AWQ mapping resolution (no kernels).

transformers 5 fuses experts into 3-D parameters; the reference (transformers 4.57) names them
per expert -- ``block_sparse_moe.experts.<e>.w1/w3/w2`` for the Mixtral family (MiniMax-M2),
``mlp.experts.<e>.{gate,up,down}_proj`` for Qwen3-MoE -- and its recipes' regexes rely on that
(recipe_Minimax-M2.1-AWQ-MixedPrec.yaml:38, :49-56)."""
import os
import warnings

import pytest
import torch

from quantizers_amd.awq import DEFAULT_MAPPINGS, resolve_mappings
from quantizers_amd.model import checkpoint_name, iter_linears
from quantizers_amd.oneshot import resolve_schemes
from quantizers_amd.recipe import parse_recipe

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _minimax(layers=2, experts=8):
    from transformers import AutoModelForCausalLM, MiniMaxM2Config
    cfg = MiniMaxM2Config(hidden_size=128, intermediate_size=64, num_hidden_layers=layers, num_attention_heads=4,
                          num_key_value_heads=2, head_dim=32, vocab_size=256, num_local_experts=experts,
                          num_experts_per_tok=2, bos_token_id=1, eos_token_id=2)
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        return AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)


def _qwen3_moe():
    from transformers import AutoModelForCausalLM, Qwen3MoeConfig
    cfg = Qwen3MoeConfig(hidden_size=128, intermediate_size=256, moe_intermediate_size=64, num_hidden_layers=1,
                         num_attention_heads=4, num_key_value_heads=2, head_dim=32, vocab_size=256, num_experts=4,
                         num_experts_per_tok=2)
    return AutoModelForCausalLM.from_config(cfg, dtype=torch.bfloat16)


def test_checkpoint_name():
    assert checkpoint_name("model.layers.3.mlp.experts", "minimax_m2") == "model.layers.3.block_sparse_moe.experts"
    assert checkpoint_name("model.layers.3.mlp", "mixtral") == "model.layers.3.block_sparse_moe"
    assert checkpoint_name("model.layers.3.mlp.gate", "qwen3_moe") == "model.layers.3.mlp.gate"
    assert checkpoint_name("model.layers.3.mlpx.a", "minimax_m2") == "model.layers.3.mlpx.a"


def test_minimax_expert_names_and_views():
    m = _minimax()
    refs = {r.name: r for r in iter_linears(m)}
    assert len(refs) == 2 * (4 + 8 * 3) + 1
    w1 = refs["model.layers.1.block_sparse_moe.experts.5.w1"]
    w3 = refs["model.layers.1.block_sparse_moe.experts.5.w3"]
    w2 = refs["model.layers.1.block_sparse_moe.experts.5.w2"]
    gu = m.model.layers[1].mlp.experts.gate_up_proj.data
    # w1 = gate rows (first half of gate_up_proj), w3 = up rows (second half), w2 = down_proj
    assert w1.weight.data_ptr() == gu[5, :64].data_ptr() and w1.weight.shape == (64, 128)
    assert w3.weight.data_ptr() == gu[5, 64:].data_ptr()
    assert w2.weight.data_ptr() == m.model.layers[1].mlp.experts.down_proj.data[5].data_ptr()


def test_minimax_recipe_targets():
    m = _minimax()
    mods = parse_recipe(os.path.join(ROOT, "configs/recipes/minimax_awq_mixedprec.yaml"))
    sch = resolve_schemes(m, mods)
    assert len(sch) == 2 * (4 + 24)
    a = sch["model.layers.0.block_sparse_moe.experts.7.w2"][0].weights
    assert (a.num_bits, a.type, a.group_size) == (4, "int", 32)
    assert sch["model.layers.0.self_attn.o_proj"][0].weights.type == "float"


def test_minimax_awq_resolution():
    m = _minimax()
    mods = parse_recipe(os.path.join(ROOT, "configs/recipes/minimax_awq_mixedprec.yaml"))
    q = {n: s.weights for n, (s, _) in resolve_schemes(m, mods).items()}
    res = resolve_mappings(m.model.layers[0], "model.layers.0", mods[0].mappings, q, "minimax_m2")
    by = {r.smooth_name: r for r in res}
    # v_proj -> o_proj dropped for GQA (D9); 1 + 1 + 8 experts
    assert len(res) == 10 and "model.layers.0.self_attn.v_proj" not in by
    a = by["model.layers.0.input_layernorm"]
    assert a.parent_name == "model.layers.0.self_attn" and len(a.balance) == 3
    p = by["model.layers.0.post_attention_layernorm"]
    assert p.parent_name == "model.layers.0.block_sparse_moe" and p.parent is m.model.layers[0].mlp
    assert len(p.balance) == 16 and p.balance_names[0].endswith("experts.0.w1") and p.balance_names[8].endswith("experts.0.w3")
    e = by["model.layers.0.block_sparse_moe.experts.3.w3"]
    assert e.balance_names == ["model.layers.0.block_sparse_moe.experts.3.w2"]
    assert e.parent_kind == "linear" and e.parent_expert == 3 and e.parent is None


def test_qwen3_moe_default_mappings():
    m = _qwen3_moe()
    names = [r.name for r in iter_linears(m)]
    assert "model.layers.0.mlp.experts.3.down_proj" in names
    q = {n: None for n in names}
    res = resolve_mappings(m.model.layers[0], "model.layers.0", DEFAULT_MAPPINGS, q, "qwen3_moe")
    by = {r.smooth_name: r for r in res}
    assert by["model.layers.0.post_attention_layernorm"].parent is m.model.layers[0].mlp
    assert len(by["model.layers.0.post_attention_layernorm"].balance) == 8
    assert by["model.layers.0.mlp.experts.2.up_proj"].balance_names == ["model.layers.0.mlp.experts.2.down_proj"]
