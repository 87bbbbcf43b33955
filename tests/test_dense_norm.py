"""dense_norm.fused_rmsnorms: which modules qualify, the patch and its restore (CPU); on the GPU
qz_rmsnorm128 against the module's own forward bit for bit (scales, strided rows, the full model,
the AWQ knob)."""
import os

import pytest
import torch

import quantizers_amd.dense_norm as dn


def _qwen3(layers=2, head_dim=128):
    from transformers import Qwen3Config, Qwen3ForCausalLM
    cfg = Qwen3Config(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=layers,
                      num_attention_heads=4, num_key_value_heads=2, head_dim=head_dim, max_position_embeddings=256)
    torch.manual_seed(0)
    m = Qwen3ForCausalLM(cfg).to(torch.bfloat16)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if n.endswith("norm.weight"):
                p.copy_((torch.rand_like(p.float()) * 1.5 + 0.25).to(p.dtype))
    return m


def test_qualifies_and_restores():
    m = _qwen3()
    norms = [mod for mod in m.modules() if type(mod).__name__ == "Qwen3RMSNorm"]
    assert norms and all(dn.qualifies(mod) for mod in norms)
    assert not dn.qualifies(m.model.layers[0].mlp)
    ids = torch.randint(0, 512, (1, 16), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        want = m(ids).logits
        with dn.fused_rmsnorms(m) as n:
            assert n == len(norms) and all("forward" in mod.__dict__ for mod in norms)
            got = m(ids).logits  # CPU: the modules' own forwards
        assert all("forward" not in mod.__dict__ for mod in norms)
    assert torch.equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [1e-3, 1.0, 40.0])
def test_rmsnorm128_bit_identical(cuda, scale):
    from transformers.models.qwen3.modeling_qwen3 import Qwen3RMSNorm
    from quantizers_amd import ops
    norm = Qwen3RMSNorm(128, eps=1e-6).to(cuda).to(torch.bfloat16)
    g = torch.Generator(device=cuda).manual_seed(int(scale * 1000))
    with torch.no_grad():
        norm.weight.copy_((torch.rand(128, generator=g, device=cuda) * 2).to(torch.bfloat16))
        x = (torch.randn(4099, 8, 128, generator=g, device=cuda) * scale).to(torch.bfloat16)
        x.view(-1)[::997] = 0.0
        x[7] = 0.0  # an all-zero row: rsqrt(eps)
        want = norm(x)
        got = ops.rmsnorm128(x, norm.weight, norm.variance_epsilon)
        assert torch.equal(got.view(torch.int16), want.view(torch.int16))
        wide = (torch.randn(1001, 3, 160, generator=g, device=cuda) * scale).to(torch.bfloat16)
        xs = wide[..., 16:144]  # rows of 128 at a row stride of 160
        assert torch.equal(ops.rmsnorm128(xs, norm.weight, norm.variance_epsilon).view(torch.int16),
                           norm(xs).view(torch.int16))


@pytest.mark.gpu
def test_fused_rmsnorms_model_bit_identical(cuda):
    m = _qwen3().to(cuda)
    ids = torch.randint(0, 512, (3, 64), generator=torch.Generator().manual_seed(2)).to(cuda)
    dn._OK.clear()
    with torch.no_grad():
        want = m(ids).logits
        with dn.fused_rmsnorms(m):
            got1 = m(ids).logits
            got2 = m(ids).logits
    assert dn._OK.get(torch.device(cuda)) is True
    assert torch.equal(got1.view(torch.int32), want.view(torch.int32))
    assert torch.equal(got2.view(torch.int32), want.view(torch.int32))


@pytest.mark.gpu
def test_fused_norm_knob_awq_bit_identical(cuda, monkeypatch):
    """QZ_FUSED_NORM on / off: the AWQ pass on a dense Qwen3 with 128-wide head norms gives the same
    loss histories and parameters."""
    from test_oneshot_gpu import ROOT, _calib, _eq
    from quantizers_amd.oneshot import oneshot
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml")
    out = {}
    for on in (True, False):
        monkeypatch.setattr(dn, "FUSED_NORM", on)
        dn._OK.clear()
        m = _qwen3().to(cuda)
        oneshot(m, recipe, dataset=_calib(n=5, vocab=512), max_seq_length=64)
        out[on] = (m.awq_report, {n: p.detach().clone() for n, p in m.named_parameters()})
    (r1, p1), (r0, p0) = out[True], out[False]
    assert r1.keys() == r0.keys()
    for layer in r1:
        for smooth, r in r1[layer].items():
            assert r.get("history") == r0[layer][smooth].get("history"), (layer, smooth)
    for n in p1:
        _eq(p1[n], p0[n], n)
