"""D15 on the CPU: moe_eager.fast_eager (two grouped GEMMs + k ordered bf16 adds) is bit-identical
to transformers' eager fused-experts forward (the reference's 4.57 per-expert loop), and the
eager_experts context patches and restores every experts module."""
import pytest
import torch

import quantizers_amd.moe_eager as me


def _models():
    from test_oneshot_gpu import _minimax, _qwen3_moe
    return {"qwen3_moe": _qwen3_moe, "minimax": _minimax}


@pytest.mark.parametrize("arch", ["qwen3_moe", "minimax"])
@pytest.mark.parametrize("tokens,k", [(300, 2), (64, 1), (1, 2)])
def test_fast_eager_bit_identical(arch, tokens, k):
    m = _models()[arch]()
    ex = next(mod for mod in m.modules() if me.eager_forward(mod) is not None)
    g = torch.Generator().manual_seed(tokens)
    x = torch.randn(tokens, ex.gate_up_proj.shape[-1], generator=g).to(torch.bfloat16)
    w, idx = torch.topk(torch.rand(tokens, ex.num_experts, generator=g).softmax(-1), k, dim=-1)
    w = (w / w.sum(-1, keepdim=True)).to(torch.bfloat16)
    with torch.no_grad():
        got = me.fast_eager(ex, x, idx, w)
        want = me.eager_forward(ex)(ex, x, idx, w)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


def test_context_patches_and_restores():
    m = _models()["qwen3_moe"]()
    mods = [mod for mod in m.modules() if me.eager_forward(mod) is not None]
    assert mods and all("forward" not in mod.__dict__ for mod in mods)
    ids = torch.randint(0, 256, (1, 16))
    with torch.no_grad(), me.eager_experts(m) as n:
        assert n == len(mods) and all("forward" in mod.__dict__ for mod in mods)
        m(ids)
        m(ids)  # second call: the verified fast path
        assert all(me.FastEagerExperts.checked.values())
    assert all("forward" not in mod.__dict__ for mod in mods)


@pytest.mark.parametrize("arch", ["qwen3_moe", "minimax"])
@pytest.mark.parametrize("tokens,k", [(300, 2), (1, 2)])
def test_planned_eager_bit_identical(arch, tokens, k):
    """The fixed-routing form (host expert bounds from one plan, one GEMM per routed expert) is
    bit-identical to the eager forward, and one plan serves repeated forwards with new expert
    weights (the AWQ grid writes its fake-quantized weights into the parameters in place)."""
    m = _models()[arch]()
    ex = next(mod for mod in m.modules() if me.eager_forward(mod) is not None)
    g = torch.Generator().manual_seed(tokens + 7)
    x = torch.randn(tokens, ex.gate_up_proj.shape[-1], generator=g).to(torch.bfloat16)
    w, idx = torch.topk(torch.rand(tokens, ex.num_experts, generator=g).softmax(-1), k, dim=-1)
    w = (w / w.sum(-1, keepdim=True)).to(torch.bfloat16)
    with torch.no_grad():
        plan = me._plan(ex, idx)
        for step in range(2):
            got = me.planned_eager(ex, x, idx, w, plan)
            want = me.eager_forward(ex)(ex, x, idx, w)
            assert torch.equal(got.view(torch.int16), want.view(torch.int16)), step
            ex.gate_up_proj.mul_(1.5)  # new weights, same routing


def test_fixed_routing_context_uses_plans():
    """Inside fixed_routing the patched experts forward takes the planned form (checked once
    against the grouped form) and equals the forward outside the context."""
    m = _models()["qwen3_moe"]()
    ids = torch.randint(0, 256, (1, 16), generator=torch.Generator().manual_seed(3))
    with torch.no_grad(), me.eager_experts(m):
        want = m(ids).logits
        m(ids)
        with me.fixed_routing():
            got1 = m(ids).logits
            got2 = m(ids).logits
            assert me._FIXED  # plans were recorded
        assert me._FIXED is None
        assert all(me.FastEagerExperts.planned_checked.values())
    assert torch.equal(got1, want) and torch.equal(got2, want)
