"""Third-party pin of the MXFP4 on-disk encoding.

compressed-tensors (where the reference's arithmetic lives) is absent, but the image ships an
independent OCP-MX decoder: transformers' gpt-oss MXFP4 loader
(``transformers/integrations/mxfp4.py``: ``FP4_VALUES`` and ``_convert_moe_packed_tensors``:
E2M1 LUT, even element in the LOW nibble, E8M0 scale = 2^(byte - 127)).  Decoding the committed
MXFP4 golden fixture (which the HIP kernel reproduces bit-exactly, tests/test_golden.py) with
that decoder must give the oracle's fake-quantized weight, element for element: this pins the
nibble order, the E2M1 code table and the E8M0 bias to a third-party implementation.
"""
import os

import pytest
import torch
from safetensors.torch import load_file

import ct_torch as ct

mxfp4 = pytest.importorskip("transformers.integrations.mxfp4")

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _tf_decode(packed: torch.Tensor, scale: torch.Tensor, group: int = 32) -> torch.Tensor:
    """[N, K/2] uint8 codes + [N, K/32] E8M0 bytes -> bf16 [N, K] via transformers' decoder."""
    n, half = packed.shape
    blocks = packed.reshape(1, n, half * 2 // group, group // 2)
    out = mxfp4._convert_moe_packed_tensors(blocks, scale.reshape(1, n, -1), dtype=torch.bfloat16)
    return out.transpose(1, 2).reshape(n, half * 2)  # the decoder returns [1, K, N]


def test_fp4_value_table_matches_transformers():
    lut = [float(v) for v in mxfp4.FP4_VALUES]
    assert lut[:8] == list(ct.FP4_GRID)
    assert lut[8:] == [-v for v in ct.FP4_GRID]


@pytest.mark.parametrize("name", ["w_gauss", "w_edge"])
def test_mxfp4_golden_decodes_to_oracle_fake_quant(name):
    a = ct.QArgs(num_bits=4, type="float", group_size=32, scale_dtype="e8m0")
    w = load_file(os.path.join(HERE, "inputs.safetensors"))[name]
    gold = load_file(os.path.join(HERE, "mxfp4_g32.safetensors"))
    packed, scale = gold[f"{name}.weight_packed"], gold[f"{name}.weight_scale"]
    mn, mx = ct.observe_minmax(w, a)
    s, zp = ct.calculate_qparams(mn, mx, a)
    assert torch.equal(s, scale)  # the fixture's scale bytes are the oracle's
    expect = ct.fake_quantize(w, s, zp, a)
    got = _tf_decode(packed, scale)
    assert got.dtype == expect.dtype == torch.bfloat16
    # -0 codes decode to -0.0 in both; compare bit patterns
    assert torch.equal(got.view(torch.int16), expect.view(torch.int16))


def test_mxfp4_random_weight_roundtrip():
    g = torch.Generator().manual_seed(7)
    w = (torch.randn(64, 1024, generator=g) * 0.05).to(torch.bfloat16)
    w[3, 64:96] = 0  # one all-zero group (scale byte 0)
    a = ct.QArgs(num_bits=4, type="float", group_size=32, scale_dtype="e8m0")
    out = ct.compress_weight(w, a)
    mn, mx = ct.observe_minmax(w, a)
    s, zp = ct.calculate_qparams(mn, mx, a)
    got = _tf_decode(out["weight_packed"], out["weight_scale"])
    assert torch.equal(got.view(torch.int16), ct.fake_quantize(w, s, zp, a).view(torch.int16))
