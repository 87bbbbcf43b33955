"""The two CPU restatements (torch op sequence vs plain C) agree bit for bit."""
import pytest
import torch

import ct_torch as ct
import qref

CASES = [
    ct.QArgs(), ct.QArgs(group_size=32), ct.QArgs(symmetric=False), ct.QArgs(symmetric=False, group_size=32),
    ct.QArgs(num_bits=8), ct.QArgs(num_bits=8, symmetric=False), ct.QArgs(num_bits=2, group_size=32),
    ct.QArgs(num_bits=3, symmetric=False, group_size=64),
    ct.QArgs(num_bits=8, type="float", group_size=32), ct.QArgs(num_bits=8, type="float", group_size=128),
    ct.QArgs(num_bits=8, type="float", strategy="block", block_structure=(32, 128)),
    ct.QArgs(num_bits=8, type="float", strategy="channel"), ct.QArgs(num_bits=8, type="float", strategy="tensor"),
    ct.QArgs(num_bits=4, type="float", group_size=32, scale_dtype="e8m0"),
    ct.QArgs(num_bits=4, type="float", group_size=16, strategy="tensor_group", scale_dtype="fp8"),
    ct.QArgs(strategy="channel"), ct.QArgs(strategy="tensor"), ct.QArgs(strategy="channel", symmetric=False),
]


def _eq(a, b):
    if a.dtype == torch.float8_e4m3fn:
        a, b = a.view(torch.uint8), b.view(torch.uint8)
    if a.dtype == torch.bfloat16:
        a, b = a.view(torch.int16), b.view(torch.int16)
    assert a.shape == b.shape and torch.equal(a, b)


@pytest.mark.parametrize("a", CASES, ids=lambda a: f"{a.type}{a.num_bits}-{a.strategy}-{a.group_size}-sym{a.symmetric}")
@pytest.mark.parametrize("seed", [0, 1])
def test_restatements_agree(a, seed):
    g = torch.Generator().manual_seed(seed)
    w = torch.randn(64, 512, generator=g) * (0.02 if seed == 0 else 3.0)
    w[5, :64] = 0
    w[7, 3] = 40.0
    w = w.to(torch.bfloat16)
    r1 = ct.compress_weight(w, a)
    r2 = qref.compress_weight(w, a)
    for k, v in r1.items():
        _eq(v, r2[k])


def test_fused_c_leg_matches():
    g = torch.Generator().manual_seed(0)
    w = (torch.randn(128, 1024, generator=g) * 0.02).to(torch.bfloat16)
    for gs in (32, 128):
        p, s = qref.int_sym_group_pack(w, 4, gs)
        r = ct.compress_weight(w, ct.QArgs(group_size=gs))
        _eq(p, r["weight_packed"])
        _eq(s, r["weight_scale"])


def test_fp4_nan_code():
    """D17: an NVFP4 slice whose |w| maximum is so small that its global scale overflows to inf
    divides its zero elements 0 / 0; both restatements encode that NaN as code 0 (of either sign
    of zero), and agree on the rest of the slice."""
    g = torch.Generator().manual_seed(3)
    w = (torch.randn(16, 64, generator=g) * 2.0 ** -122).to(torch.bfloat16)
    w[0, :4] = 0.0
    w[1, :4] = -0.0
    a = ct.QArgs(num_bits=4, type="float", group_size=16, strategy="tensor_group", scale_dtype="fp8")
    r1, r2 = ct.compress_weight(w, a), qref.compress_weight(w, a)
    assert torch.isinf(r1["weight_global_scale"]).all()
    for k, v in r1.items():
        _eq(v, r2[k])
    codes = r1["weight_packed"]
    assert (codes[0, :2] == 0).all() and (codes[1, :2] == 0).all()
