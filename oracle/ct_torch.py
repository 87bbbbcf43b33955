"""CPU oracle — op-for-op restatement of the reference's weight-quantization arithmetic.

TEST INFRASTRUCTURE ONLY.  Nothing in ``quantizers_amd/`` imports this module; only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use it,
and only as the checker / the timed CPU baseline, never as the product path.

What it restates
----------------
The reference (mratsim/quantizers) performs no quantization arithmetic of its own: the
per-linear quantize step happens inside ``llmcompressor.oneshot`` (``scripts/do_oneshot.py:179-187``)
and ``model.save_pretrained(save_compressed=True)`` (``scripts/do_oneshot.py:197``), i.e. in
the third-party packages ``compressed-tensors>=0.13.0`` and ``llmcompressor>=0.9.0``
(``pyproject.toml:10-11``; the author's run used compressed-tensors
``0.13.1.dev0+g797d301``, ``scripts/recombine_weights_MiniMax-M2.1.py:133``).  Neither package
is vendored in /root/reference nor installed in this image, so this file restates their
published algorithm as the SAME sequence of PyTorch CPU ops (so every bf16 intermediate is
rounded exactly where compressed-tensors materialises a bf16 tensor).

PARITY STATUS: **parity unpinned** against the third-party code (it cannot run here and the
reference's own tests hold no vectors for this path).  The restatement is
pinned instead by (1) hand-derived known-answer tests (tests/test_oracle_kat.py), (2) an
independent plain-C restatement (oracle/quant_ref.c) that must agree bit-for-bit, and (3) the
on-disk tensor contract the reference itself encodes
(``scripts/recombine_weights_MiniMax-M2.1.py:54-65,82-134``).  Every point where the
third-party semantics are uncertain is a numbered decision D1..D11.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Optional, Tuple

import torch

BF16_EPS = torch.finfo(torch.bfloat16).eps  # 2**-7 (D1: zero scale -> finfo(scale dtype).eps)
FP8_MAX = 448.0
FP4_MAX = 6.0
FP4_GRID = (0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0)


@dataclass
class QArgs:
    """Mirror of compressed-tensors ``QuantizationArgs`` fields used by the reference's recipes
    (``configs/recipes/recipe_awq_w4a16.yaml:16-24``, ``recipe_mixed_fp8_int4.yaml:9-24``,
    ``recipe_Minimax-M2.1-AWQ-MixedPrec.yaml:24-48``)."""

    num_bits: int = 4
    type: str = "int"  # "int" | "float"
    symmetric: bool = True
    strategy: str = "group"  # tensor | channel | group | block | tensor_group
    group_size: Optional[int] = 128
    block_structure: Optional[Tuple[int, int]] = None
    scale_dtype: Optional[str] = None  # None (= weight dtype) | "fp8" (NVFP4) | "e8m0" (MXFP4)
    observer: str = "memoryless_minmax"

    @property
    def is_mx(self) -> bool:
        return self.type == "float" and self.num_bits == 4 and self.scale_dtype == "e8m0"

    @property
    def is_fp4(self) -> bool:
        return self.type == "float" and self.num_bits == 4


# ----------------------------------------------------------------------------------------
# calculate_range  ([3P] compressed_tensors.quantization.utils.helpers.calculate_range)
# ----------------------------------------------------------------------------------------
def calculate_range(a: QArgs) -> Tuple[torch.Tensor, torch.Tensor]:
    if a.type == "int":
        bit_range = 2 ** a.num_bits
        return torch.tensor(-bit_range / 2), torch.tensor(bit_range / 2 - 1)
    if a.num_bits == 8:
        return torch.tensor(-FP8_MAX), torch.tensor(FP8_MAX)
    if a.num_bits == 4:
        return torch.tensor(-FP4_MAX), torch.tensor(FP4_MAX)
    raise ValueError(f"unsupported float num_bits {a.num_bits}")


# ----------------------------------------------------------------------------------------
# observer: memoryless min/max over the calibration layout ([3P] llmcompressor observers +
# flatten_for_calibration)
# ----------------------------------------------------------------------------------------
def flatten_for_calibration(w: torch.Tensor, a: QArgs) -> torch.Tensor:
    """Returns a view [..., n_groups, elems] whose last dim is reduced by the observer."""
    n, k = w.shape
    if a.strategy == "tensor":
        return w.reshape(1, 1, -1)
    if a.strategy == "channel":
        return w.reshape(n, 1, k)
    if a.strategy in ("group", "tensor_group"):
        g = a.group_size
        if k % g:
            raise ValueError(f"tensor column shape must be divisible by group_size {g}")
        return w.reshape(n, k // g, g)
    if a.strategy == "block":
        bh, bw = a.block_structure
        if n % bh or k % bw:
            raise ValueError("Block quantization requires exact division")
        return w.reshape(n // bh, bh, k // bw, bw).transpose(1, 2).reshape(n // bh, k // bw, bh * bw)
    raise ValueError(a.strategy)


def observe_minmax(w: torch.Tensor, a: QArgs) -> Tuple[torch.Tensor, torch.Tensor]:
    f = flatten_for_calibration(w, a)
    mn = torch.amin(f, dim=-1)
    mx = torch.amax(f, dim=-1)
    if a.strategy == "tensor":
        mn, mx = mn.reshape(1), mx.reshape(1)
    return mn, mx


def moving_average_minmax(mn, mx, past_mn, past_mx, averaging_constant: float = 0.01):
    """``minmax`` observer (D7): lerp with the previous observation, in the weight dtype."""
    if past_mn is None:
        return mn, mx
    mn = past_mn + averaging_constant * (mn - past_mn)
    mx = past_mx + averaging_constant * (mx - past_mx)
    return mn, mx


# ----------------------------------------------------------------------------------------
# MX helpers ([3P] compressed_tensors mxfp4 utils)
# ----------------------------------------------------------------------------------------
def round_to_power_2(x: torch.Tensor) -> torch.Tensor:
    """bf16 bit trick: add half a mantissa step (0x40) then keep sign|exponent (0xFF80)."""
    assert x.dtype == torch.bfloat16
    xi = x.view(torch.int16).to(torch.int32) & 0xFFFF
    r = torch.bitwise_and(xi + (1 << 6), ((1 << 9) - 1) << 7) & 0xFFFF
    r = torch.where(r >= 0x8000, r - 0x10000, r)
    return r.to(torch.int16).view(torch.bfloat16)


def generate_mx_scales(amax: torch.Tensor) -> torch.Tensor:
    """E8M0 exponent byte = 127 + floor(log2(round_to_power_2(amax))) - 2 (emax of E2M1).
    round_to_power_2 leaves a pure power of two whose bf16 exponent field E gives
    floor(log2) = E - 127, so the byte is E - 2.  D6/D11: clamped to [0, 254]; an all-zero
    group (E = 0, log2 = -inf) -> 0."""
    e = (round_to_power_2(amax).view(torch.int16).to(torch.int32) >> 7) & 0xFF
    return torch.clamp(e - 2, 0, 254).to(torch.uint8)


def mx_scale_to_dense(e8: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    return (2.0 ** (e8.to(torch.int32) - 127).to(torch.float)).to(dtype)


# ----------------------------------------------------------------------------------------
# calculate_qparams ([3P] compressed_tensors.quantization.utils.helpers)
# ----------------------------------------------------------------------------------------
def calculate_qparams(mn: torch.Tensor, mx: torch.Tensor, a: QArgs,
                      global_scale: Optional[torch.Tensor] = None):
    """Returns (scale, zero_point).  scale dtype: weight dtype (D3), fp8 for NVFP4, uint8 E8M0 for MX.
    zero_point: int8 (sym -> zeros)."""
    mn = torch.min(mn, torch.zeros_like(mn))
    mx = torch.max(mx, torch.zeros_like(mx))
    bit_min, bit_max = calculate_range(a)
    bit_range = bit_max - bit_min
    if a.symmetric:
        amax = torch.max(torch.abs(mn), torch.abs(mx))
        if a.is_mx:
            return generate_mx_scales(amax), torch.zeros(amax.shape, dtype=torch.int8)
        scales = amax / (float(bit_range) / 2)
        zps = torch.zeros(scales.shape, dtype=mn.dtype)
    else:
        if a.is_fp4:
            raise NotImplementedError("Asymmetric Quantization is not supported for FP4")
        scales = (mx - mn) / float(bit_range)
        zps = bit_min - (mn / scales)
        zps = torch.clamp(zps, bit_min, bit_max)
    if global_scale is not None:
        scales = global_scale * scales  # f32 * bf16 -> f32
    if a.scale_dtype == "fp8":
        scales = torch.clamp(scales, -FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).to(scales.dtype)
        eps = 0.125  # _get_dtype_eps(float8_e4m3fn)
    else:
        eps = torch.finfo(scales.dtype).eps
    scales = torch.where(scales == 0, torch.tensor(eps, dtype=scales.dtype), scales)
    if a.scale_dtype == "fp8":
        scales = scales.to(torch.float8_e4m3fn)
    # D10: round(NaN) -> int8 is 0 on x86 torch; the build defines it as 0.
    zps = torch.round(zps).to(torch.int8)
    return scales, zps


def generate_gparam(mn: torch.Tensor, mx: torch.Tensor) -> torch.Tensor:
    """NVFP4 global scale ([3P] generate_gparam): (448*6)/tensor_absmax computed in the weight dtype (D5)."""
    mn = torch.min(mn, torch.zeros_like(mn))
    mx = torch.max(mx, torch.zeros_like(mx))
    amax = torch.max(torch.abs(mn), torch.abs(mx))
    return (FP8_MAX * FP4_MAX / amax).to(torch.float32).reshape([1])


# ----------------------------------------------------------------------------------------
# rounding / casting ([3P] round_to_quantized_type_args, FP4_E2M1_DATA.cast_to_fp4)
# ----------------------------------------------------------------------------------------
def cast_to_fp4(x: torch.Tensor) -> torch.Tensor:
    sign = torch.sign(x)
    x = torch.abs(x)
    x[(x >= 0.0) & (x <= 0.25)] = 0.0
    x[(x > 0.25) & (x < 0.75)] = 0.5
    x[(x >= 0.75) & (x <= 1.25)] = 1.0
    x[(x > 1.25) & (x < 1.75)] = 1.5
    x[(x >= 1.75) & (x <= 2.5)] = 2.0
    x[(x > 2.5) & (x < 3.5)] = 3.0
    x[(x >= 3.5) & (x <= 5.0)] = 4.0
    x[x > 5.0] = 6.0
    return x * sign


def round_to_quantized_type(t: torch.Tensor, a: QArgs, qmin, qmax) -> torch.Tensor:
    orig = t.dtype
    t = torch.clamp(t, qmin, qmax)
    if a.type == "float":
        r = t.to(torch.float8_e4m3fn) if a.num_bits == 8 else cast_to_fp4(t)
    else:
        r = torch.round(t)
    return r.to(orig)


def _group_view(x: torch.Tensor, a: QArgs):
    """Expand per-group params to the element layout (mirrors _process_quantization)."""
    n, k = x.shape
    if a.strategy in ("group", "tensor_group"):
        return x.reshape(n, k // a.group_size, a.group_size), (lambda p: p.unsqueeze(-1))
    if a.strategy == "channel":
        return x, (lambda p: p.reshape(n, 1))
    if a.strategy == "tensor":
        return x, (lambda p: p.reshape(1, 1))
    if a.strategy == "block":
        bh, bw = a.block_structure
        xv = x.reshape(n // bh, bh, k // bw, bw)
        return xv, (lambda p: p.reshape(n // bh, 1, k // bw, 1))
    raise ValueError(a.strategy)


def _dense_scale(scale: torch.Tensor, a: QArgs, x_dtype, global_scale):
    if a.is_mx:
        return mx_scale_to_dense(scale, x_dtype)
    if global_scale is not None:
        return scale.to(torch.float32) / global_scale  # fp8 / f32 -> f32 (D5)
    return scale


def quantize(x: torch.Tensor, scale: torch.Tensor, zp: Optional[torch.Tensor], a: QArgs,
             dtype=None, global_scale=None) -> torch.Tensor:
    """[3P] compressed_tensors quantize -> _process_quantization -> _quantize."""
    qmin, qmax = calculate_range(a)
    xv, ex = _group_view(x, a)
    s = ex(_dense_scale(scale, a, x.dtype, global_scale))
    scaled = xv / s
    if zp is not None and not a.is_mx:
        scaled = scaled + ex(zp).to(x.dtype)
    q = round_to_quantized_type(scaled, a, qmin, qmax)
    if dtype is not None:
        q = q.to(dtype)
    return q.reshape(x.shape)


def dequantize(q: torch.Tensor, scale: torch.Tensor, zp: Optional[torch.Tensor], a: QArgs,
               dtype=None, global_scale=None) -> torch.Tensor:
    """[3P] _dequantize: (q - zp) * scale in the scale dtype."""
    qv, ex = _group_view(q, a)
    s = ex(_dense_scale(scale, a, torch.bfloat16, global_scale))
    d = qv.to(s.dtype)
    if zp is not None and not a.is_mx and not a.symmetric:
        d = d - ex(zp).to(s.dtype)
    d = d * s
    if dtype is not None:
        d = d.to(dtype)
    return d.reshape(q.shape)


def fake_quantize(x, scale, zp, a: QArgs, global_scale=None):
    q = quantize(x, scale, zp, a, dtype=None, global_scale=global_scale)
    return dequantize(q, scale, zp if not a.symmetric else None, a, global_scale=global_scale).to(x.dtype)


# ----------------------------------------------------------------------------------------
# packers ([3P] pack_to_int32 / pack_fp4_to_uint8)
# ----------------------------------------------------------------------------------------
def pack_to_int32(value: torch.Tensor, num_bits: int, packed_dim: int = 1) -> torch.Tensor:
    if value.dtype is not torch.int8:
        raise ValueError("Tensor must be quantized to torch.int8 before packing")
    if num_bits > 8:
        raise ValueError("Packing is only supported for less than 8 bits")
    offset = 1 << (num_bits - 1)
    value = (value + offset).to(torch.uint8)
    pack_factor = 32 // num_bits
    if packed_dim == 0:
        value = value.transpose(0, 1)
    rows, cols = value.shape
    padded = math.ceil(cols / pack_factor) * pack_factor
    if padded != cols:
        value = torch.nn.functional.pad(value, (0, padded - cols))
    reshaped = value.reshape(rows, padded // pack_factor, pack_factor).to(torch.int32)
    shifts = torch.arange(pack_factor, dtype=torch.int32) * num_bits
    packed = (reshaped << shifts).sum(dim=2, dtype=torch.int32)
    if packed_dim == 0:
        packed = packed.transpose(0, 1)
    return packed.contiguous()


def unpack_from_int32(packed: torch.Tensor, num_bits: int, shape, packed_dim: int = 1) -> torch.Tensor:
    pack_factor = 32 // num_bits
    mask = (1 << num_bits) - 1
    if packed_dim == 0:
        packed = packed.transpose(0, 1)
    shifts = torch.arange(pack_factor, dtype=torch.int32) * num_bits
    u = (packed.unsqueeze(-1) >> shifts) & mask
    u = u.reshape(packed.shape[0], -1)
    n = shape[1] if packed_dim == 1 else shape[0]
    u = u[:, :n]
    if packed_dim == 0:
        u = u.transpose(0, 1)
    return (u - (1 << (num_bits - 1))).to(torch.int8).contiguous()


def pack_fp4_to_uint8(x: torch.Tensor) -> torch.Tensor:
    m, n = x.shape
    grid = torch.tensor(FP4_GRID, dtype=x.dtype)
    idx = torch.argmin(torch.abs(torch.abs(x).unsqueeze(-1) - grid), dim=-1)
    idx = idx + (torch.signbit(x).to(torch.long) << 3)
    idx[torch.isnan(x)] = 0  # D17: a NaN's sign bit is platform-defined (x86 0/0 is negative)
    idx = idx.reshape(-1, 2)
    return (idx[:, 0] | (idx[:, 1] << 4)).to(torch.uint8).reshape(m, n // 2)


# ----------------------------------------------------------------------------------------
# compressor-level: one weight -> the tensors written to disk (the names are
# pinned by scripts/recombine_weights_MiniMax-M2.1.py:54-65)
# ----------------------------------------------------------------------------------------
def compress_weight(w: torch.Tensor, a: QArgs) -> dict:
    out = {}
    gs = None
    if a.strategy == "tensor_group":
        tmn, tmx = w.amin().reshape(1), w.amax().reshape(1)
        gs = generate_gparam(tmn, tmx)
        out["weight_global_scale"] = gs
    mn, mx = observe_minmax(w, a)
    scale, zp = calculate_qparams(mn, mx, a, global_scale=gs)
    if a.type == "int":
        q = quantize(w, scale, zp, a, dtype=torch.int8)
        out["weight_packed"] = pack_to_int32(q, a.num_bits)
        out["weight_scale"] = scale
        out["weight_shape"] = torch.tensor(w.shape)
        if not a.symmetric and a.strategy in ("group", "channel"):
            out["weight_zero_point"] = pack_to_int32(zp.reshape(scale.shape), a.num_bits, packed_dim=0)
    elif a.num_bits == 8:
        out["weight"] = quantize(w, scale, zp, a, dtype=torch.float8_e4m3fn)
        out["weight_scale"] = scale
    else:
        q = quantize(w, scale, zp, a, global_scale=gs)
        out["weight_packed"] = pack_fp4_to_uint8(q)
        out["weight_scale"] = scale
    return out


# ----------------------------------------------------------------------------------------
# AWQ pieces ([3P] llmcompressor.modifiers.awq)
# ----------------------------------------------------------------------------------------
def awq_accumulate_mean(x: torch.Tensor, prev=None):
    """D8: the build accumulates Σ|x| in fp32 (llmcompressor uses the activation dtype)."""
    s = x.reshape(-1, x.shape[-1]).abs().float().sum(0)
    n = x.reshape(-1, x.shape[-1]).shape[0]
    if prev is None:
        return s, n
    return prev[0] + s, prev[1] + n


def awq_layer_means(weights, a: QArgs) -> torch.Tensor:
    """w_mean: mean over rows of |W| / (group absmax + 1e-6), bf16 elementwise, f64 sum."""
    total = 0
    acc = 0
    for w in weights:
        n, k = w.shape
        g = {"tensor": w.numel(), "channel": k}.get(a.strategy, a.group_size)
        if a.strategy == "block":
            g = k  # D9b: block-strategy balance layers normalised per row
        v = w.reshape(-1, g)
        v = v.abs() / (v.abs().amax(dim=1, keepdim=True) + 1e-6)
        v = v.reshape(n, k)
        total += n
        acc = acc + v.sum(0, dtype=torch.float64)
    return acc / total


def awq_grid_scales(x_mean: torch.Tensor, w_mean: torch.Tensor, ratio: float, duo: bool = True):
    """One point of the 20-ratio grid, in fp32 (D8b)."""
    x_mean = x_mean.float()
    w_mean = w_mean.float()
    if duo:
        s = (x_mean.pow(ratio) / (w_mean.pow(1 - ratio) + 1e-4)).clamp(min=1e-4)
    else:
        s = x_mean.pow(ratio).clamp(min=1e-4)
    s = s / (s.max() * s.min()).sqrt()
    s[torch.isinf(s)] = 1
    s[torch.isnan(s)] = 1
    return s


def awq_fake_quant_scaled(w: torch.Tensor, s: torch.Tensor, a: QArgs) -> torch.Tensor:
    """W' = Q(W*s)/s with the balance layer's own scheme (bf16 products, f32 scales)."""
    ws = (w.float() * s.float().view(1, -1)).to(w.dtype)
    gs = None
    if a.strategy == "tensor_group":
        gs = generate_gparam(ws.amin().reshape(1), ws.amax().reshape(1))
    mn, mx = observe_minmax(ws, a)
    scale, zp = calculate_qparams(mn, mx, a, global_scale=gs)
    fq = fake_quantize(ws, scale, zp, a, global_scale=gs)
    return (fq.float() / s.float().view(1, -1)).to(w.dtype)


# ----------------------------------------------------------------------------------------
# D8, the literal reading of SURVEY A.6 ("accumulation dtype = activation dtype"): every AWQ
# statistic, grid scale and scaled weight in the weight / activation dtype (bf16), the loss an f32
# sum per calibration batch.  Since round 5 this is the oracle of the product's DEFAULT reading
# (awq_dtype="bf16"; the fp32 reading's oracle is awq_* above).  Op order as llmcompressor's
# _accumulate_mean / _compute_layer_means / _compute_best_scale / _compute_loss ([3P], unpinned).
#
# Device semantics: llmcompressor's sequential pipeline runs each layer -- and so
# the activation hook's and _compute_layer_means' tensor ops -- on the accelerator.  The one op whose
# bits depend on that is the division of a bf16 tensor by a Python number: torch's CPU kernel
# divides (bf16(f32(a) / f32(n))), its GPU kernel multiplies by the f32 reciprocal of the scalar
# (bf16(f32(a) * (1.0f / f32(n))), BinaryDivTrueKernel's CPU-scalar case).  device_division=True
# restates the GPU form, the product's; False the CPU form.  Every other op here (bf16 x scalar
# product, bf16 adds, pow, clamp, amax / amin) rounds f32 arithmetic to bf16 identically on both.
# ----------------------------------------------------------------------------------------
def div_scalar_bf16(t: torch.Tensor, n, device_division: bool) -> torch.Tensor:
    """bf16 tensor / Python number as torch computes it on the GPU (reciprocal product,
    ``device_division``) or on the CPU (true division)."""
    if not device_division:
        return t / n
    import numpy as np
    inv = float(np.float32(1.0) / np.float32(n))
    return (t.float() * inv).to(t.dtype)


def awq_accumulate_mean_literal(x: torch.Tensor, prev=None, device_division: bool = False):
    """Running mean of |x| over tokens in x's dtype: (prev_mean * prev_n + sum) / (prev_n + n),
    every op rounded to bf16 (the per-batch sum accumulates in f32 inside torch, rounded once)."""
    inp = x.reshape(-1, x.shape[-1]).abs()
    return awq_running_mean_from_sums_literal([(inp.sum(0), inp.shape[0])], prev, device_division)


def awq_running_mean_from_sums_literal(parts, prev=None, device_division: bool = True):
    """_accumulate_mean over per-batch column sums [(sum, n), ...] in batch order: each sum
    rounded once to bf16 (a bf16 tensor's ``sum(0)`` accumulates in f32 and rounds once; an f32
    sum given here, e.g. the absmean kernel's, is rounded here), then (prev_mean * prev_n + sum) /
    (prev_n + n) in bf16.  Returns (mean, count); batches without tokens are skipped."""
    for s, n in parts:
        if n == 0:
            continue
        s = s.to(torch.bfloat16)
        if prev is None:
            prev = (div_scalar_bf16(s, n, device_division), n)
        else:
            pm, pc = prev
            prev = (div_scalar_bf16(pm * pc + s, pc + n, device_division), pc + n)
    return prev


def awq_layer_means_literal(weights, a: QArgs, device_division: bool = False) -> torch.Tensor:
    """w_mean in the weight dtype: per layer a bf16 column sum, summed across layers in bf16,
    divided by the row count in bf16."""
    parts = []
    for w in weights:
        n, k = w.shape
        g = {"tensor": w.numel(), "channel": k}.get(a.strategy, a.group_size)
        if a.strategy == "block":
            g = k
        v = w.reshape(-1, g)
        v = (v.abs() / (v.abs().amax(dim=1, keepdim=True) + 1e-6)).reshape(n, k)
        parts.append((v.sum(0), n))
    return awq_layer_means_from_sums_literal(parts, device_division)


def awq_layer_means_from_sums_literal(parts, device_division: bool = True) -> torch.Tensor:
    """_compute_layer_means' combination of per-layer column sums [(sum, rows), ...] in the
    mapping's balance order: each sum rounded once to bf16 (torch's bf16 ``sum(0)`` rounds its f32
    accumulation once; the w_mean kernel's f64 sum is rounded here), added in bf16, divided by the
    total row count in bf16."""
    acc, total = None, 0
    for s, n in parts:
        s = s.to(torch.bfloat16)
        acc = s if acc is None else acc + s
        total += n
    return div_scalar_bf16(acc, total, device_division)


def awq_grid_scales_literal(x_mean: torch.Tensor, w_mean: torch.Tensor, ratio: float, duo: bool = True):
    """One grid point with x_mean / w_mean in bf16: every op of the formula rounds to bf16."""
    if duo:
        s = (x_mean.pow(ratio) / (w_mean.pow(1 - ratio) + 1e-4)).clamp(min=1e-4)
    else:
        s = x_mean.pow(ratio).clamp(min=1e-4)
    s = s / (s.max() * s.min()).sqrt()
    s[torch.isinf(s)] = 1
    s[torch.isnan(s)] = 1
    return s


def awq_fake_quant_scaled_literal(w: torch.Tensor, s: torch.Tensor, a: QArgs) -> torch.Tensor:
    """Q(W*s)/s with a bf16 scale vector: W.mul_(s) and the division in bf16."""
    ws = w * s.view(1, -1)
    gs = None
    if a.strategy == "tensor_group":
        gs = generate_gparam(ws.amin().reshape(1), ws.amax().reshape(1))
    mn, mx = observe_minmax(ws, a)
    scale, zp = calculate_qparams(mn, mx, a, global_scale=gs)
    return fake_quantize(ws, scale, zp, a, global_scale=gs) / s.view(1, -1)
