"""Third-party pins of the on-disk encodings (MXFP4, FP8 group / block / channel, int4 packed words).

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


# ---------------------------------------------------------------------------------------------
# FP8 (group / block / channel) and MXFP4 through a second outside decoder: transformers'
# fine-grained FP8 dequantizer (``transformers/integrations/finegrained_fp8.py``,
# ``Fp8Dequantize._dequantize_one``).  It derives the block from the scale grid (rows / scale
# rows x cols / scale cols), multiplies e4m3 codes (or E2M1 nibbles, low nibble first, with
# E8M0 scales 2^(byte - 127)) by the block's scale in f32 and rounds to bf16 -- which is
# compressed-tensors' dequantize for these schemes, so decoding the committed fixtures must give
# the oracle's fake-quantized weight bit for bit.  This pins the e4m3 code bytes, the scale
# layout (row-major [N / bh, K / bw]) and the block orientation to outside code.
fg = pytest.importorskip("transformers.integrations.finegrained_fp8")

FP8_CASES = [("fp8_g32.safetensors", ct.QArgs(num_bits=8, type="float", group_size=32), "weight"),
             ("fp8_block128.safetensors", ct.QArgs(num_bits=8, type="float", strategy="block",
                                                   block_structure=(128, 128)), "weight"),
             ("fp8_channel.safetensors", ct.QArgs(num_bits=8, type="float", strategy="channel"), "weight")]


def _fg_decode(codes: torch.Tensor, scale: torch.Tensor) -> torch.Tensor:
    return fg.Fp8Dequantize(None)._dequantize_one(codes, scale, output_dtype=torch.bfloat16)


@pytest.mark.parametrize("fixture,a,key", FP8_CASES, ids=["fp8_g32", "fp8_block128", "fp8_channel"])
@pytest.mark.parametrize("name", ["w_gauss", "w_edge"])
def test_fp8_golden_decodes_to_oracle_fake_quant(fixture, a, key, name):
    w = load_file(os.path.join(HERE, "inputs.safetensors"))[name]
    gold = load_file(os.path.join(HERE, fixture))
    codes = gold[f"{name}.{key}"].view(torch.float8_e4m3fn)
    scale = gold[f"{name}.weight_scale"]
    mn, mx = ct.observe_minmax(w, a)
    s, zp = ct.calculate_qparams(mn, mx, a)
    assert torch.equal(s.reshape(scale.shape).view(torch.int16), scale.view(torch.int16))
    expect = ct.fake_quantize(w, s, zp, a)
    got = _fg_decode(codes, scale)
    assert torch.equal(got.view(torch.int16), expect.view(torch.int16))


@pytest.mark.parametrize("name", ["w_gauss", "w_edge"])
def test_mxfp4_golden_decodes_with_finegrained_dequant(name):
    a = ct.QArgs(num_bits=4, type="float", group_size=32, scale_dtype="e8m0")
    w = load_file(os.path.join(HERE, "inputs.safetensors"))[name]
    gold = load_file(os.path.join(HERE, "mxfp4_g32.safetensors"))
    packed, scale = gold[f"{name}.weight_packed"], gold[f"{name}.weight_scale"]
    mn, mx = ct.observe_minmax(w, a)
    s, zp = ct.calculate_qparams(mn, mx, a)
    got = _fg_decode(packed.view(torch.int8), scale.view(torch.uint8))
    assert torch.equal(got.view(torch.int16), ct.fake_quantize(w, s, zp, a).view(torch.int16))


# ---------------------------------------------------------------------------------------------
# int4 pack-quantized words through a third outside decoder: transformers' Metal affine
# dequantizer (``transformers/integrations/metal_quantization.py``,
# ``_affine_dequantize_tensor``: element i of a 32-bit word at bits 4i, word k of a row holding
# columns 8k..8k+7, value = u * scale + bias per group).  compressed-tensors' symmetric int4 value
# (u - 8) * s is that affine form with bias = -8 s (exact in f32), the asymmetric one
# (u - 8 - zp) * s with bias = (-8 - zp) s; the zero points (packed along dim 0, D2) are unpacked
# by the same routine on the transposed words.  Pins the nibble order, the word layout and the +8
# offset of pack_to_int32 to outside code.
metal = pytest.importorskip("transformers.integrations.metal_quantization")


def _metal_unpack_codes(words: torch.Tensor) -> torch.Tensor:
    """[R, W] int32 words -> [R, 8 W] unsigned nibbles via the Metal decoder (scale 1, bias 0)."""
    r, wcols = words.shape  # one group per row: scale 1, bias 0
    return metal._affine_dequantize_tensor(words, torch.ones(r, 1), torch.zeros(r, 1), wcols * 8, 4)


@pytest.mark.parametrize("fixture,group,sym", [("int4_sym_g128", 128, True), ("int4_sym_g32", 32, True),
                                               ("int4_asym_g128", 128, False), ("int4_asym_g32", 32, False)])
@pytest.mark.parametrize("name", ["w_gauss", "w_edge"])
def test_int4_packed_golden_decodes_with_metal_affine_dequant(fixture, group, sym, name):
    a = ct.QArgs(num_bits=4, group_size=group, symmetric=sym)
    w = load_file(os.path.join(HERE, "inputs.safetensors"))[name]
    gold = load_file(os.path.join(HERE, f"{fixture}.safetensors"))
    packed, scale = gold[f"{name}.weight_packed"], gold[f"{name}.weight_scale"].float()
    n = packed.shape[0]
    if sym:
        zp = torch.zeros_like(scale)
    else:  # zero points packed along dim 0: unpack the transposed words with the same decoder
        zpk = gold[f"{name}.weight_zero_point"]
        zp = (_metal_unpack_codes(zpk.t().contiguous()).t()[:n] - 8)
    got = metal._affine_dequantize_tensor(packed, scale, (-8.0 - zp) * scale, group, 4).to(torch.bfloat16)
    mn, mx = ct.observe_minmax(w, a)
    s, z = ct.calculate_qparams(mn, mx, a)
    expect = ct.fake_quantize(w, s, z, a)
    # the decoders cannot produce -0 (u * s + b); the oracle's fake-quant keeps torch.round's sign
    assert torch.equal(got.float(), expect.float())


def test_fp4_encode_matches_torchao_encoder():
    """compressed-tensors' cast_to_fp4 threshold ladder (oracle) == torchao's E2M1 encoder
    (``_f32_to_floatx_unpacked``, vendored in torch.testing._internal.common_quantized, written
    outside this repository and outside compressed-tensors) on every finite bf16 value, the codes
    packed by torch's ``pack_uint4`` in the oracle's nibble order (even element in the low
    nibble).  Exact -0.0 is the one documented difference (D11: torch.sign(-0.) = 0 gives code 0;
    torchao keeps the sign bit); values beyond +-6 saturate in both."""
    import sys
    import types
    stub = "expecttest" not in sys.modules
    if stub:  # torch's test utilities import this test-runner package (absent here) at module level;
        try:  # nothing used below touches it
            import expecttest  # noqa: F401
            stub = False
        except ImportError:
            sys.modules["expecttest"] = types.SimpleNamespace(TestCase=object)
    try:
        cq = pytest.importorskip("torch.testing._internal.common_quantized")
    finally:
        if stub:
            sys.modules.pop("expecttest", None)
    bits = torch.arange(65536, dtype=torch.int32).to(torch.int16).view(torch.bfloat16)
    x = bits[torch.isfinite(bits.float())]
    x = x[~((x == 0) & torch.signbit(x.float()))]  # exact -0.0: D11
    t = torch.clamp(x.float(), -6.0, 6.0)  # round_to_quantized_type clamps before the cast
    ours = ct.pack_fp4_to_uint8(ct.cast_to_fp4(t.clone()).reshape(1, -1)[:, : t.numel() // 2 * 2])
    theirs = cq.pack_uint4(cq._f32_to_floatx_unpacked(x.float()[: t.numel() // 2 * 2].contiguous(), 2, 1))
    assert torch.equal(ours.reshape(-1), theirs.reshape(-1))
    # and the decode direction: torchao's unpacked E2M1 -> f32 table is the oracle's grid
    codes = torch.arange(16, dtype=torch.uint8)
    vals = cq._floatx_unpacked_to_f32(codes, 2, 1)
    assert vals[:8].tolist() == list(ct.FP4_GRID) and vals[8:].tolist() == [-v for v in ct.FP4_GRID]
