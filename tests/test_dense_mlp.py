"""dense_mlp.fused_mlps: which modules qualify, the patch and its restore (CPU), and on the GPU
the fused SiLU·up forward against the module's own forward, bit for bit (incl. AWQ knob check)."""
import os

import pytest
import torch
from torch import nn

import quantizers_amd.dense_mlp as dm


def _qwen3(layers=2):
    from transformers import Qwen3Config, Qwen3ForCausalLM
    cfg = Qwen3Config(vocab_size=256, hidden_size=128, intermediate_size=256, num_hidden_layers=layers,
                      num_attention_heads=4, num_key_value_heads=2, head_dim=32, max_position_embeddings=128)
    torch.manual_seed(0)
    return Qwen3ForCausalLM(cfg).to(torch.bfloat16)


def test_qualifies_and_restores():
    m = _qwen3()
    mlps = [mod for mod in m.modules() if type(mod).__name__ == "Qwen3MLP"]
    assert mlps and all(dm.qualifies(mod) for mod in mlps)
    assert not dm.qualifies(m.model.layers[0].self_attn)

    class Other(nn.Module):  # same attributes, a different forward
        def __init__(self):
            super().__init__()
            self.gate_proj, self.up_proj, self.down_proj = nn.Linear(4, 8), nn.Linear(4, 8), nn.Linear(8, 4)
            self.act_fn = nn.SiLU()

        def forward(self, x):
            return self.down_proj(self.act_fn(self.up_proj(x)) * self.gate_proj(x))
    assert not dm.qualifies(Other())
    ids = torch.randint(0, 256, (1, 16), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        want = m(ids).logits
        with dm.fused_mlps(m) as n:
            assert n == len(mlps) and all("forward" in mod.__dict__ for mod in mlps)
            got = m(ids).logits  # CPU: the composed ops
        assert all("forward" not in mod.__dict__ for mod in mlps)
    assert torch.equal(got, want)


@pytest.mark.gpu
def test_fused_mlp_bit_identical_gpu(cuda):
    """On the GPU the patched forward (qz_silu_mul between the projections) equals the module's
    own forward bit for bit, the hooks on the projections fire once each, in the same order."""
    m = _qwen3().to(cuda)
    order = []
    for name in ("gate_proj", "up_proj", "down_proj"):
        getattr(m.model.layers[0].mlp, name).register_forward_pre_hook(lambda mod, a, n=name: order.append(n))
    ids = torch.randint(0, 256, (3, 64), generator=torch.Generator().manual_seed(2)).to(cuda)
    dm._OK.clear()
    with torch.no_grad():
        want = m(ids).logits
        ref_order, order[:] = list(order), []
        with dm.fused_mlps(m):
            got1 = m(ids).logits  # first call: checked, composed result
            got2 = m(ids).logits  # fused
        assert order == ref_order * 2
    assert dm._OK.get(torch.device(cuda)) is True
    assert torch.equal(got1.view(torch.int32), want.view(torch.int32))
    assert torch.equal(got2.view(torch.int32), want.view(torch.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("rows,inter,strided", [(300, 9728, False), (257, 100, False), (64, 256, True)])
def test_silu_mul_two_inputs_bit_identical(cuda, rows, inter, strided):
    from quantizers_amd import ops
    g = torch.Generator().manual_seed(rows + inter)
    a = (torch.randn(rows, 2 * inter if strided else inter, generator=g) * 4).to(torch.bfloat16).to(cuda)
    b = (torch.randn(rows, 2 * inter if strided else inter, generator=g) * 4).to(torch.bfloat16).to(cuda)
    gate, up = (a[:, :inter], b[:, inter:]) if strided else (a, b)
    want = nn.functional.silu(gate) * up
    got = ops.silu_mul(gate, up)
    assert torch.equal(got.view(torch.int16), want.view(torch.int16))


@pytest.mark.gpu
def test_fused_mlp_knob_awq_bit_identical(cuda, monkeypatch):
    """QZ_FUSED_MLP on / off: the whole AWQ pass on a dense Qwen3 (calibration, the gate/up grid
    over the MLP parent, propagation) gives the same loss histories and parameters."""
    from test_oneshot_gpu import ROOT, _calib, _eq, _qwen3 as _q
    from quantizers_amd.oneshot import oneshot
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml")
    out = {}
    for on in (True, False):
        monkeypatch.setattr(dm, "FUSED_MLP", on)
        dm._OK.clear()
        m = _q().to(cuda)
        oneshot(m, recipe, dataset=_calib(n=5, vocab=512), max_seq_length=64)
        out[on] = (m.awq_report, {n: p.detach().clone() for n, p in m.named_parameters()})
    (r1, p1), (r0, p0) = out[True], out[False]
    assert r1.keys() == r0.keys()
    for layer in r1:
        for smooth, r in r1[layer].items():
            assert r.get("history") == r0[layer][smooth].get("history"), (layer, smooth)
    for n in p1:
        _eq(p1[n], p0[n], n)
