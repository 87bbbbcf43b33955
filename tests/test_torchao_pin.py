"""Outside code pins the oracle's integer qparam formulas (oracle/ct_torch.calculate_qparams,
fake_quantize): torch's own quantization observers (torch.ao.quantization.observer
.PerChannelMinMaxObserver / MinMaxObserver, shipped in the image's torch, not written here) compute
the same range-with-zero, symmetric divisor (qmax - qmin) / 2, asymmetric scale (max - min) /
(qmax - qmin) and zero point qmin - round(min / scale), clamped.  Evaluated in f32 (torch.ao's
arithmetic), the oracle's scales and zero points equal torch.ao's bit for bit, for int4 / int8,
symmetric / asymmetric, group / channel / tensor strategies.

torch.fake_quantize_per_channel_affine rounds x * (1 / scale) and then adds the zero point;
compressed-tensors (and the oracle, and the kernels) round x / scale + zero point: the fake-quantized
values agree except where those two forms round to different integers, and the test checks that
is the only difference.

Not pinned here: the bf16 evaluation points (D3), zero groups (D1 / D10: torch.ao clamps the scale
to eps BEFORE the zero point, compressed-tensors >= 0.12 after it, so an all-zero asymmetric group
gets zero point qmin there and 0 here), the FP8 / FP4 schemes."""
import pytest
import torch

import ct_torch as ct
from torch.ao.quantization.observer import MinMaxObserver, PerChannelMinMaxObserver


def _weights(seed=0, rows=192, cols=1024):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(rows, cols, generator=g) * (torch.rand(rows, 1, generator=g) * 0.1 + 1e-3)
    w[3] = w[3].abs()  # all-positive rows / groups: the range must still include zero
    w[5] = -w[5].abs()
    return w


def _ao(x2d, sym, qmin, qmax, per_channel=True):
    if per_channel:
        obs = PerChannelMinMaxObserver(ch_axis=0, dtype=torch.qint8, quant_min=qmin, quant_max=qmax,
                                       qscheme=torch.per_channel_symmetric if sym else torch.per_channel_affine)
    else:
        obs = MinMaxObserver(dtype=torch.qint8, quant_min=qmin, quant_max=qmax,
                             qscheme=torch.per_tensor_symmetric if sym else torch.per_tensor_affine)
    obs(x2d)
    return obs.calculate_qparams()


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("strategy", ["group", "channel", "tensor"])
def test_qparams_match_torch_ao_observers(bits, sym, strategy):
    w = _weights(seed=bits * 10 + sym)
    a = ct.QArgs(num_bits=bits, type="int", symmetric=sym, strategy=strategy, group_size=128)
    qmin, qmax = (int(v) for v in ct.calculate_range(a))
    mn, mx = ct.observe_minmax(w, a)
    s_ct, z_ct = ct.calculate_qparams(mn, mx, a)
    # the same units as torch.ao channels: one row per group / channel, the tensor as one
    x2d = {"group": w.reshape(-1, 128), "channel": w, "tensor": w}[strategy]
    s_ao, z_ao = _ao(x2d, sym, qmin, qmax, per_channel=strategy != "tensor")
    assert s_ct.dtype == torch.float32
    assert torch.equal(s_ct.reshape(-1), s_ao.reshape(-1)), "scales"
    assert torch.equal(z_ct.reshape(-1).long(), z_ao.reshape(-1).long()), "zero points"
    # fake quantization: torch's kernel rounds x * (1 / s), the oracle x / s
    fq_ct = ct.fake_quantize(w, s_ct, z_ct, a)
    sv = s_ao.reshape(-1).float()
    zv = z_ao.reshape(-1).int()
    if strategy == "tensor":
        fq_ao = torch.fake_quantize_per_tensor_affine(w, float(sv[0]), int(zv[0]), qmin, qmax)
        s_el, z_el = sv[0], zv[0].float()
        x = w
    else:
        fq_ao = torch.fake_quantize_per_channel_affine(x2d, sv, zv, 0, qmin, qmax).reshape(w.shape)
        s_el, z_el = sv[:, None], zv[:, None].float()
        x = x2d
    # compressed-tensors: round(x / s + zp); torch's kernel: round(x * (1 / s)) + zp
    q_div = torch.clamp(torch.round(x / s_el + z_el), qmin, qmax).reshape(w.shape)
    q_mul = torch.clamp(torch.round(x * (1.0 / s_el)) + z_el, qmin, qmax).reshape(w.shape)
    same = q_div == q_mul
    assert torch.equal(fq_ct[same], fq_ao[same])
    assert (~same).float().mean() < 2e-3  # the quotient forms disagree only next to a rounding tie
    assert ((q_div - q_mul).abs() <= 1).all()


@pytest.mark.parametrize("bits", [4, 8])
@pytest.mark.parametrize("sym", [True, False])
@pytest.mark.parametrize("group", [32, 128, 0])
def test_bf16_qparams_match_torch_affine_quantization(bits, sym, group):
    """D3 in bf16: torch's affine quantization primitives (torch.ao.quantization.pt2e.
    _affine_quantization._choose_qparams_affine, the torchao algorithm shipped in the image's torch)
    evaluate the qparams in the weight's dtype (bf16 min / max, bf16 scale, zero point from a bf16
    quotient), as the oracle restates compressed-tensors: group-wise (block [1, g]) and per-channel
    (g = 0: block [1, cols]) scales are bit-identical on bf16 weights, int4 / int8, symmetric /
    asymmetric, and so are the zero points except where compressed-tensors' extra bf16 rounding of
    qmin - min / s (its op order) crosses a half-integer.  eps is passed as bf16's smallest normal, so torchao's clamp touches only
    all-zero groups, which the data avoids (D1 / D10 differ there, see the module docstring)."""
    from torch.ao.quantization.pt2e._affine_quantization import _choose_qparams_affine
    w = _weights(seed=100 + bits + 2 * sym + group, rows=256, cols=2048).to(torch.bfloat16)
    strategy = "group" if group else "channel"
    a = ct.QArgs(num_bits=bits, type="int", symmetric=sym, strategy=strategy, group_size=group or None)
    qmin, qmax = (int(v) for v in ct.calculate_range(a))
    mn, mx = ct.observe_minmax(w, a)
    s_ct, z_ct = ct.calculate_qparams(mn, mx, a)
    s_ao, z_ao = _choose_qparams_affine(w, "SYMMETRIC" if sym else "ASYMMETRIC", [1, group or w.shape[1]],
                                        torch.int8, qmin, qmax, eps=torch.finfo(torch.bfloat16).tiny)
    assert s_ct.dtype == s_ao.dtype == torch.bfloat16
    assert torch.equal(s_ct.reshape(-1).view(torch.int16), s_ao.reshape(-1).view(torch.int16)), "scales"
    # zero points: torchao takes qmin - round(bf16(min / s)); compressed-tensors rounds
    # bf16(qmin - bf16(min / s)), one more bf16 rounding -- they may differ only where that rounding
    # moves the value across a half-integer (1 group in 16384 here)
    if sym:
        assert torch.equal(z_ct.reshape(-1).float(), z_ao.reshape(-1).float()), "zero points"
        return
    q = (torch.min(mn, torch.zeros_like(mn)) / s_ct).reshape(-1)
    torchao_form = qmin - torch.round(q.float())
    ct_form = torch.round((qmin - q).float())
    same = torchao_form == ct_form
    assert torch.equal(z_ct.reshape(-1).float()[same], z_ao.reshape(-1).float()[same]), "zero points"
    assert torch.equal(z_ct.reshape(-1).float(), torch.clamp(ct_form, qmin, qmax))
    assert (~same).sum() <= max(2, same.numel() // 1000)


@pytest.mark.parametrize("shape", ["group32", "group128", "channel", "block128"])
def test_bf16_fp8_scales_match_torch_affine_quantization(shape):
    """FP8-E4M3 scales (FP8 group / channel presets and FP8_BLOCK 128 x 128, the reference's mixed
    and data-free recipes): torchao's symmetric float8 qparams (amax / ((qmax - qmin) / 2) with
    qmax = 448, evaluated in bf16) equal the oracle's bf16 scales bit for bit."""
    from torch.ao.quantization.pt2e._affine_quantization import _choose_qparams_affine
    w = _weights(seed=200 + len(shape), rows=256, cols=2048).to(torch.bfloat16)
    args = {"group32": dict(strategy="group", group_size=32), "group128": dict(strategy="group", group_size=128),
            "channel": dict(strategy="channel"), "block128": dict(strategy="block", block_structure=(128, 128))}[shape]
    block = {"group32": [1, 32], "group128": [1, 128], "channel": [1, 2048], "block128": [128, 128]}[shape]
    a = ct.QArgs(num_bits=8, type="float", symmetric=True, **args)
    mn, mx = ct.observe_minmax(w, a)
    s_ct, _ = ct.calculate_qparams(mn, mx, a)
    s_ao, _ = _choose_qparams_affine(w, "SYMMETRIC", block, torch.float8_e4m3fn,
                                     eps=torch.finfo(torch.bfloat16).tiny)
    assert s_ct.dtype == s_ao.dtype == torch.bfloat16
    assert torch.equal(s_ct.reshape(-1).view(torch.int16), s_ao.reshape(-1).view(torch.int16))
