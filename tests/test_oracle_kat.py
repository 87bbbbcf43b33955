"""Known-answer tests pinning the CPU oracle (SURVEY.md §8c KATs, hand-derived).

These pin both restatements (oracle/ct_torch.py torch op sequence and oracle/quant_ref.c);
compressed-tensors itself is absent here, so parity with it is unpinned.
"""
import numpy as np
import pytest
import torch

import ct_torch as ct
import qref

BOTH = [ct.compress_weight, qref.compress_weight]


def _bf(vals, shape=None):
    t = torch.tensor(vals, dtype=torch.float32).to(torch.bfloat16)
    return t.reshape(shape) if shape else t


@pytest.mark.parametrize("impl", BOTH)
def test_absmax_maps_to_plus7_minus8(impl):
    # group of 8 (g=8): absmax element -> +7 (7.5 -> clamp 7), -absmax -> -8 (RNE(-7.5) = -8)
    w = _bf([0.75, -0.75, 0.05, -0.05, 0.15, 0.25, -0.35, 0.0], (1, 8))
    a = ct.QArgs(num_bits=4, group_size=8)
    out = impl(w, a)
    s = out["weight_scale"].float().item()
    assert s == torch.tensor(0.75 / 7.5).to(torch.bfloat16).float().item()
    q = ct.unpack_from_int32(out["weight_packed"], 4, (1, 8))[0].tolist()
    assert q[0] == 7 and q[1] == -8 and q[7] == 0
    # the middle codes follow bf16(w/s) then round-half-even (s = bf16(0.1) is not exactly 0.1)
    t = (w.float() / s).to(torch.bfloat16)
    expect = torch.round(torch.clamp(t, -8, 7)).to(torch.int8)[0].tolist()
    assert q == expect


def test_pack_kat():
    q = torch.arange(-8, 8, dtype=torch.int8).reshape(1, 16)
    p = ct.pack_to_int32(q, 4)
    assert p.tolist() == [[0x76543210, -19088744]]  # 0xFEDCBA98 as int32
    assert p[0, 0].item() == 1985229328
    out = torch.empty(1, 2, dtype=torch.int32)
    qref.lib().qref_pack_int32(qref._ptr(q), 1, 16, 4, qref._ptr(out))
    assert torch.equal(out, p)
    assert torch.equal(ct.unpack_from_int32(p, 4, (1, 16)), q)


def test_pack_dim0_zero_points():
    zp = torch.tensor([[-8, 7], [0, 1], [3, -3]], dtype=torch.int8)
    p = ct.pack_to_int32(zp, 4, packed_dim=0)
    assert p.shape == (1, 2)
    col0 = (0) | (8 << 4) | (11 << 8)
    col1 = (15) | (9 << 4) | (5 << 8)
    assert p.tolist() == [[col0, col1]]


def test_e4m3_clamp_and_exhaustive_table():
    # clamp 449 -> 448, 464 -> 448 (after clamp no NaN)
    a = ct.QArgs(num_bits=8, type="float", strategy="tensor")
    w = _bf([448.0, 449.0, 464.0, -500.0, 1.0], (1, 5))
    mn, mx = ct.observe_minmax(w, a)
    s, z = ct.calculate_qparams(mn, mx, a)
    q = ct.quantize(w, torch.ones_like(s), None, a, dtype=torch.float8_e4m3fn)
    assert q.view(torch.uint8).tolist()[0][:4] == [0x7E, 0x7E, 0x7E, 0xFE]
    # exhaustive bf16 -> e4m3 (finite, |x| <= 448) via the C restatement == torch cast
    bits = torch.arange(0, 65536, dtype=torch.int32)
    bits = torch.where(bits >= 32768, bits - 65536, bits).to(torch.int16)
    x = bits.view(torch.bfloat16)
    keep = torch.isfinite(x.float()) & (x.float().abs() <= 448)
    x = x[keep].reshape(1, -1)
    a = ct.QArgs(num_bits=8, type="float", strategy="tensor")
    ref = torch.clamp(x, -448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
    # divide by scale 1: build a group whose absmax is 448 so s = 1
    x2 = torch.cat([x, _bf([448.0], (1, 1))], 1)
    out = qref.compress_weight(x2, a)
    assert out["weight_scale"].float().item() == 1.0
    assert torch.equal(out["weight"].view(torch.uint8)[:, :-1], ref)


def test_zero_group_scale_is_bf16_eps():
    w = torch.zeros(2, 32, dtype=torch.bfloat16)
    for impl in BOTH:
        out = impl(w, ct.QArgs(num_bits=4, group_size=32))
        assert out["weight_scale"].float().unique().tolist() == [0.0078125]
        assert out["weight_packed"].unique().tolist() == [0x88888888 - (1 << 32)]
        out = impl(w, ct.QArgs(num_bits=4, group_size=32, symmetric=False))
        assert out["weight_scale"].float().unique().tolist() == [0.0078125]


def test_mx_kats():
    a = ct.QArgs(num_bits=4, type="float", group_size=32, scale_dtype="e8m0")
    w = torch.zeros(2, 32)
    w[0, 0] = 1.0   # amax 1.0 -> E 127 -> byte 125 -> 2^-2 ; 1.0/0.25 = 4 -> code 6
    w[1, 0] = 1.5   # amax 1.5 -> rounds up to 2 -> byte 126 -> 0.5 ; 1.5/0.5 = 3 -> code 5
    w[1, 1] = -0.1  # -0.2 -> |.| <= .25 -> -0 -> code 8
    w = w.to(torch.bfloat16)
    for impl in BOTH:
        out = impl(w, a)
        assert out["weight_scale"][:, 0].tolist() == [125, 126]
        assert out["weight_packed"][0, 0].item() & 15 == 6
        assert out["weight_packed"][1, 0].item() == (5 | (8 << 4))


def test_nvfp4_kat():
    a = ct.QArgs(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="fp8")
    w = torch.zeros(1, 16)
    w[0, 0] = 6.0
    w[0, 1] = -3.0
    w = w.to(torch.bfloat16)
    for impl in BOTH:
        out = impl(w, a)
        # gs = bf16(bf16(1/6) * 2688) = 448 ; s8 = e4m3(448 * 1) = 0x7E ; 6/1 -> code 7 ; -3 -> 0xD
        assert out["weight_global_scale"].item() == 448.0
        assert out["weight_scale"].view(torch.uint8).item() == 0x7E
        assert out["weight_packed"][0, 0].item() == (7 | (0xD << 4))


def test_fp4_cast_thresholds():
    x = torch.tensor([0.25, 0.26, 0.75, 1.25, 1.26, 1.75, 2.5, 2.6, 3.5, 5.0, 5.1, -0.1, -0.0, 0.0])
    got = ct.cast_to_fp4(x.clone())
    assert got.tolist() == [0.0, 0.5, 1.0, 1.0, 1.5, 2.0, 2.0, 3.0, 4.0, 4.0, 6.0, -0.0, 0.0, 0.0]
    assert torch.signbit(got[11]) and not torch.signbit(got[12])
