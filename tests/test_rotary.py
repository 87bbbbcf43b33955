"""rotary.fused_rotary: which transformers modules get the swap, and its restore (CPU); on the GPU
qz_rotary128 against apply_rotary_pos_emb bit for bit (transposed heads, broadcast cos / sin, the
full model, the AWQ knob)."""
import os

import pytest
import torch

import quantizers_amd.rotary as rt
from quantizers_amd.patching import same_code


def test_swap_scope_and_restore():
    import transformers.models.minimax_m2.modeling_minimax_m2 as mm
    import transformers.models.qwen3.modeling_qwen3 as q3
    from test_dense_norm import _qwen3
    assert same_code(q3.apply_rotary_pos_emb, rt.apply_rotary_pos_emb) and same_code(q3.rotate_half, rt.rotate_half)
    assert not same_code(mm.apply_rotary_pos_emb, rt.apply_rotary_pos_emb)  # partial rotary: not swapped
    m = _qwen3()
    orig = q3.apply_rotary_pos_emb
    ids = torch.randint(0, 512, (1, 16), generator=torch.Generator().manual_seed(1))
    with torch.no_grad():
        want = m(ids).logits
        with rt.fused_rotary(m) as n:
            assert n == 1 and q3.apply_rotary_pos_emb is not orig
            got = m(ids).logits  # CPU: the original function
        assert q3.apply_rotary_pos_emb is orig
    assert torch.equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("B,H,T,bcast", [(2, 8, 300, False), (1, 32, 2048, True), (3, 4, 17, True)])
def test_rotary128_bit_identical(cuda, B, H, T, bcast):
    from quantizers_amd import ops
    g = torch.Generator(device=cuda).manual_seed(B * 1000 + T)
    proj = (torch.randn(B, T, H, 128, generator=g, device=cuda) * 3).to(torch.bfloat16)
    x = proj.transpose(1, 2)  # [B, H, T, 128] as the attention forward hands it over
    ang = torch.rand(1 if bcast else B, T, 64, generator=g, device=cuda) * 50
    emb = torch.cat((ang, ang), dim=-1)
    cos, sin = emb.cos().to(torch.bfloat16), emb.sin().to(torch.bfloat16)
    want_q, want_k = rt.apply_rotary_pos_emb(x, x, cos, sin)
    got = ops.rotary128(x, cos, sin)
    assert got.stride() == want_q.stride()
    assert torch.equal(got.view(torch.int16), want_q.view(torch.int16))


@pytest.mark.gpu
def test_fused_rotary_model_bit_identical(cuda):
    from test_dense_norm import _qwen3
    m = _qwen3().to(cuda)
    ids = torch.randint(0, 512, (3, 64), generator=torch.Generator().manual_seed(2)).to(cuda)
    rt._OK.clear()
    with torch.no_grad():
        want = m(ids).logits
        with rt.fused_rotary(m):
            got1 = m(ids).logits
            got2 = m(ids).logits
    assert rt._OK.get(torch.device(cuda)) is True
    assert torch.equal(got1.view(torch.int32), want.view(torch.int32))
    assert torch.equal(got2.view(torch.int32), want.view(torch.int32))


@pytest.mark.gpu
def test_fused_rotary_knob_awq_bit_identical(cuda, monkeypatch):
    from test_dense_norm import _qwen3
    from test_oneshot_gpu import ROOT, _calib, _eq
    from quantizers_amd.oneshot import oneshot
    recipe = os.path.join(ROOT, "configs", "recipes", "awq_w4a16_g32.yaml")
    out = {}
    for on in (True, False):
        monkeypatch.setattr(rt, "FUSED_ROTARY", on)
        rt._OK.clear()
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
