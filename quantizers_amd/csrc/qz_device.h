// qz_device.h -- gfx950 device arithmetic shared by the quantize / AWQ kernels.
//
// Bit-exactness contract: every value compressed-tensors materialises
// as a bf16 tensor is rounded here with round-to-nearest-even to bf16 (v_cvt_pk_bf16_f32) at
// the same point; scalar-by-tensor quotients use IEEE-correct f32 division; per-element
// bf16/bf16 quotients use x * rcp(s), which is provably equal to bf16(x / s) for 8-bit
// operands (proof in DESIGN.md §Numerics "rcp lemma", exhaustively tested in
// tests/test_rcp_lemma.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/quantizers_amd.h"

namespace qz {

// --------------------------------------------------------------------------- kinds
enum Kind : int { K_INT = 0, K_FP8 = 1, K_MX = 2, K_NV = 3, K_FP4 = 4 };

// Host+device view of the per-call quantization constants.
struct QP {
  float qmin, qmax;   // calculate_range
  float half_range;   // (qmax - qmin) / 2  (symmetric scale divisor)
  float range;        // qmax - qmin        (asymmetric scale divisor)
  float inv_half;     // f32(1 / half_range), correctly rounded (host)
  float inv_range;    // f32(1 / range)
  float magic;        // 2^23 - qmin: t + magic has RNE(t) - qmin in its low mantissa bits
  int bits;
  int sym;
  int kind;
};

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
// round an f32 result to bf16 (RNE, v_cvt_pk_bf16_f32) and widen back
__device__ __forceinline__ float bfr(float f) { return bf2f(f2bf(f)); }

// 16-B write-through (sc1) global store: the line does not stay dirty in the XCD's L2, so the
// end-of-kernel release has nothing to write back (MI355X_MICROARCH.md: 16-B sc1 store ~ plain;
// plain 16-B stores measured no faster).  The trailing s_nop keeps the compiler's next
// instruction off the data VGPRs until the store has read them (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void st16_wt(void* p, const uint4 v) {
  typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t d = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1\n\ts_nop 1" ::"v"(p), "v"(d) : "memory");
}

// Output stores of the streaming quantize kernels: non-temporal through most of a launch, but the
// workgroups that write the launch's LAST QZ_WT_TAIL_BYTES of outputs store write-through (sc1,
// 16 B per lane): a non-temporal store leaves its line dirty in the XCD's L2, and what is still
// dirty when the launch ends is written back by the end-of-kernel release, on the critical path
// (MI355X_MICROARCH.md price list, "boundary": + bytes / 6 TB/s); write-through stores all the way
// cost 2-4 % on multi-GB launches (profiles/r05d_tune_plan.log).  Workgroups are ranked by linear
// id (blockIdx.y * gridDim.x + blockIdx.x), the order they are dispatched in.  The int4 group path
// takes a 32 MiB tail: the whole-model plan (5 launches) 1366.0 -> 1358.0 us; 64 / 128 / 256 MiB
// tails and whole launches were slower in the plan although faster launch by launch in isolation
// (profiles/r05e_tune_plan.log, r05f_tune_plan.log).  The FP8_BLOCK strip kernel takes none
// (qz_block.hip).
// The tail is taken only by launches whose outputs are at least QZ_WT_MIN_OUT_BYTES: below that the
// "tail" would be the whole launch (every workgroup pays the quad gather and 1 lane in 4 stores),
// which cost the one-weight [11008, 4096] launch (22.5 MB of codes) 0.4-0.5 us in the bench's
// pattern (12 rotating weights into 100 fresh output sets: 20.92 / 21.08 / 20.64 us with it, 20.46
// / 20.56 / 20.44 us gated, on three boxes, rocprof medians of 700 launches; profiles/r06a-d_wt_ab.log).
// It wins only when a launch rewrites the outputs the previous one wrote (19.56-20.16 vs 20.28-20.44
// us), which no product path does.  Fractional tails (1/8, 1/4, 1/2 of the outputs), 4-B sc1 and
// default-policy code stores for such launches measured no better.  Every launch of the headline
// plan writes >= 90 MiB, so it keeps its tail (1354.1 / 1381.3 / 1390 us per step, gated vs
// 1354.1 / 1385.0 / 1392 ungated).
#ifndef QZ_WT_TAIL_BYTES
#define QZ_WT_TAIL_BYTES (32ll << 20)
#endif
#ifndef QZ_WT_MIN_OUT_BYTES
#define QZ_WT_MIN_OUT_BYTES (2 * QZ_WT_TAIL_BYTES)
#endif
__device__ __forceinline__ bool wt_tail(uint32_t wt_from) {
  return blockIdx.y * gridDim.x + blockIdx.x >= wt_from;
}
// first workgroup of the write-through tail of a launch of `wgs` workgroups writing `out_bytes`
// (0xffffffff = no tail)
inline uint32_t wt_tail_from(int64_t wgs, int64_t out_bytes, int64_t tail_bytes = QZ_WT_TAIL_BYTES) {
  if (out_bytes < QZ_WT_MIN_OUT_BYTES) return 0xffffffffu;
  if (wgs <= 0 || out_bytes <= 0 || wgs >= 0xffffffffll || tail_bytes <= 0) return 0xffffffffu;
  const int64_t per = (out_bytes + wgs - 1) / wgs;
  const int64_t tail = (tail_bytes + per - 1) / per;
  return (uint32_t)(tail >= wgs ? 0 : wgs - tail);
}

// torch.clamp: NaN propagates
__device__ __forceinline__ float clamp_t(float x, float lo, float hi) {
  return (x != x) ? x : fminf(fmaxf(x, lo), hi);
}

// order-preserving float <-> uint32 keys (atomicMin/Max on floats)
__device__ __forceinline__ uint32_t f2key(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float key2f(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// ------------------------------------------------------------- float8_e4m3fn (OCP)
// RNE encode of a finite value with |x| <= 448 given as a bf16 bit pattern.
__device__ __forceinline__ uint32_t bf16_to_e4m3(uint32_t b) {
  uint32_t sign = (b >> 8) & 0x80u;
  uint32_t E = (b >> 7) & 0xffu, m7 = b & 0x7fu;
  uint32_t code;
  if (E >= 121u) {  // e4m3 normal range (>= 2^-6)
    uint32_t v = ((E - 120u) << 7) | m7;
    v += 0x7u + ((v >> 4) & 1u);
    code = v >> 4;
  } else {  // e4m3 subnormal: units of 2^-9
    uint32_t mant = E ? (128u + m7) : m7;
    uint32_t sh = E ? (125u - E) : 124u;  // value = mant * 2^(E-134) (E>0) ; units 2^-9
    if (sh > 24u) sh = 24u;
    uint32_t half = 1u << (sh - 1u);
    code = (mant + half - 1u + ((mant >> sh) & 1u)) >> sh;
  }
  return sign | code;
}
// f32 -> e4m3 for a value that is not necessarily bf16 (NVFP4 scales): RNE, |x| <= 448
__device__ __forceinline__ uint32_t f32_to_e4m3(float f) {
  uint32_t u = __float_as_uint(f);
  uint32_t sign = (u >> 24) & 0x80u;
  float a = fabsf(f);
  if (a < 0.015625f) {
    float n = __builtin_rintf(a * 512.0f);
    return sign | (uint32_t)n;
  }
  uint32_t au = __float_as_uint(a);
  uint32_t v = ((((au >> 23) & 0xffu) - 120u) << 23) | (au & 0x7fffffu);  // 4-bit exp field
  v += 0x7ffffu + ((v >> 20) & 1u);
  return sign | (v >> 20);
}
__device__ __forceinline__ float e4m3_to_f32(uint32_t c) {
  uint32_t s = (c & 0x80u) << 24;
  uint32_t e = (c >> 3) & 0xfu, m = c & 7u;
  float v;
  if (e == 0) v = (float)m * 0.001953125f;  // m * 2^-9
  else v = __uint_as_float(((e + 120u) << 23) | (m << 20));
  return __uint_as_float(__float_as_uint(v) | s);
}

// ------------------------------------------------------------------ FP4 E2M1
// FP4_E2M1_DATA.cast_to_fp4 thresholds on |x|; sign bit from sign(x) (x<0 -> 0x8, even when
// the magnitude rounds to 0).  A NaN passes no threshold test: code 0 (D17)
__device__ __forceinline__ uint32_t fp4_code(float x) {
  float a = fabsf(x);
  uint32_t idx = (a > 0.25f) + (a >= 0.75f) + (a > 1.25f) + (a >= 1.75f) + (a > 2.5f) +
                 (a >= 3.5f) + (a > 5.0f);
  return idx | ((x < 0.0f) ? 8u : 0u);
}
__device__ __forceinline__ float fp4_value(uint32_t code) {
  const float mag[8] = {0.f, 0.5f, 1.f, 1.5f, 2.f, 3.f, 4.f, 6.f};
  float v = mag[code & 7u];
  return (code & 8u) ? -v : v;
}

// 2^e for e in [-127, 127] (2^-127 is the f32 subnormal 0x00400000)
__device__ __forceinline__ float mx_pow2(int e) {
  return e >= -126 ? __uint_as_float((uint32_t)(e + 127) << 23) : __uint_as_float(0x00400000u);
}

// bf16(a / b) for a bf16 value a and a divisor b of <= 8 significant bits, given rb within
// 1 ulp of 1/b: equal to the IEEE quotient rounded to bf16 whenever the quotient is normal
// (rcp lemma); tiny / huge / non-finite quotients take the IEEE division.
__device__ __forceinline__ float bf16_quot(float a, float b, float rb) {
  float q = a * rb;
  const float aq = fabsf(q);
  if (__builtin_expect(!(aq >= 0x1.0p-120f && aq <= 0x1.0p+120f), 0)) q = a / b;
  return bfr(q);
}

// ------------------------------------------------------- cross-lane integer reductions
// xor-butterfly reduction over groups of L consecutive lanes.  L <= 16 uses DPP (VALU
// cross-lane, no LDS round trip): quad_perm [1,0,3,2], quad_perm [2,3,0,1], row_half_mirror,
// row_mirror; wider groups fall back to ds_bpermute shuffles.  Reductions run on uint32 keys
// (order-preserving images of the floats) so no NaN canonicalisation is needed and the DPP
// move folds into v_max_u32_dpp / v_min_u32_dpp.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);  // full EXEC: every source lane valid
}
template <int L>
__device__ __forceinline__ uint32_t grp_max_u(uint32_t v) {
  if (L >= 2) v = max(v, dpp<0xB1>(v));
  if (L >= 4) v = max(v, dpp<0x4E>(v));
  if (L >= 8) v = max(v, dpp<0x141>(v));
  if (L >= 16) v = max(v, dpp<0x140>(v));
#pragma unroll
  for (int m = 16; m < L; m <<= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m, 64));
  return v;
}
template <int L>
__device__ __forceinline__ uint32_t grp_min_u(uint32_t v) {
  if (L >= 2) v = min(v, dpp<0xB1>(v));
  if (L >= 4) v = min(v, dpp<0x4E>(v));
  if (L >= 8) v = min(v, dpp<0x141>(v));
  if (L >= 16) v = min(v, dpp<0x140>(v));
#pragma unroll
  for (int m = 16; m < L; m <<= 1) v = min(v, (uint32_t)__shfl_xor((int)v, m, 64));
  return v;
}
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_max_u16(uint32_t a, uint32_t b) {
  return __builtin_bit_cast(uint32_t, __builtin_elementwise_max(__builtin_bit_cast(u16x2, a), __builtin_bit_cast(u16x2, b)));
}


// ------------------------------------------------------------- per-group params
struct GP {
  float s;      // dense scale (bf16 value, 2^k for MX, f32 for NV)
  float rs;     // reciprocal used by the per-element fast quotient
  float zp;     // zero point as float (exact integer)
  uint32_t sbits;  // stored scale bits (bf16 / e4m3 / e8m0)
  bool fast;    // x * rs is exact-equivalent (see header)
};

// calculate_qparams for one group from its observed min/max (bf16 values as f32).
// gs: NVFP4 global scale (K_NV only).
// mx_is_absmax: symmetric group whose caller passes max(|min|, |max|) as mx (mn unused)
__device__ __forceinline__ GP group_params(const QP& p, float mn, float mx, float gs, bool mx_is_absmax = false) {
  GP g;
  float lo = fminf(mn, 0.f), hi = fmaxf(mx, 0.f);
  g.zp = 0.f;
  if (p.kind == K_MX) {
    float am = mx_is_absmax ? mx : fmaxf(fabsf(lo), fabsf(hi));
    uint32_t b = f2bf(am);
    uint32_t e = ((b + 0x40u) >> 7) & 0xffu;  // round_to_power_2 -> exponent field
    int byte = (int)e - 2;
    byte = byte < 0 ? 0 : (byte > 254 ? 254 : byte);
    g.sbits = (uint32_t)byte;
    // 2^(byte-127) and its reciprocal 2^(127-byte); both f32-representable
    g.s = mx_pow2(byte - 127);
    g.rs = mx_pow2(127 - byte);
    g.fast = true;
    return g;
  }
  float s;
  if (p.sym) {
    float am = mx_is_absmax ? mx : fmaxf(fabsf(lo), fabsf(hi));
    s = (am == 0.f) ? 0.f : bf16_quot(am, p.half_range, p.inv_half);
  } else {
    const float rng = bfr(hi - lo);
    s = (rng == 0.f) ? 0.f : bf16_quot(rng, p.range, p.inv_range);
    float t = (s == 0.f || lo == 0.f) ? lo / s : bf16_quot(lo, s, __builtin_amdgcn_rcpf(s));
    g.zp = clamp_t(bfr(p.qmin - t), p.qmin, p.qmax);
    // D10: NaN zp -> 0.  "+ 0.0f" turns rint's -0 into +0: the reference's zero point is an
    // int8, and a -0 zp would flip the sign of an exactly-zero fake-quant result
    g.zp = (g.zp != g.zp) ? 0.f : __builtin_rintf(g.zp) + 0.0f;
  }
  if (p.kind == K_NV) {
    float s32 = gs * s;
    uint32_t s8 = f32_to_e4m3(clamp_t(s32, -448.f, 448.f));
    float sf = e4m3_to_f32(s8);
    if (sf == 0.f) { s8 = 0x20u; sf = 0.125f; }  // eps of float8_e4m3fn
    g.sbits = s8;
    g.s = sf / gs;  // _quantize: scale / global_scale (f32)
    // f32 quotient x / s: the fast kernel forms x * rs and falls back to the IEEE division
    // only when x * rs is within a few ulps of an E2M1 rounding boundary (encode_store)
    g.rs = __builtin_amdgcn_rcpf(g.s);  // approximate (1 ulp): only steers the fast path
    g.fast = (g.s >= 0x1.0p-100f) && (g.s <= 0x1.0p+100f);
    return g;
  }
  if (s == 0.f) s = 0.0078125f;  // D1: finfo(bf16).eps
  g.s = s;
  g.sbits = f2bf(s);
  g.rs = __builtin_amdgcn_rcpf(s);
  g.fast = (s >= 0x1.0p-125f) && (s <= 0x1.0p+125f);
  return g;
}

// calculate_qparams of a symmetric group with a bf16 scale (int / FP8 / native-FP4 kinds) from
// its absmax: the same result as group_params(p, -am, am, 0, true) with the common case
// branch-light -- s = bf16(am * (1 / half_range)) when that product is a normal in
// [2^-120, 2^120] (one unsigned compare on its bits; rcp lemma), else the general routine
// (zero groups, extreme magnitudes)
__device__ __forceinline__ GP group_params_sym(const QP& p, float am) {
  const float q = am * p.inv_half;
  if (__builtin_expect(__float_as_uint(q) - 0x03800000u <= 0x78000000u, 1)) {
    GP g;
    g.sbits = f2bf(q);
    g.s = bf2f((uint16_t)g.sbits);
    g.rs = __builtin_amdgcn_rcpf(g.s);
    g.zp = 0.f;
    g.fast = true;
    return g;
  }
  return group_params(p, -am, am, 0.f, true);
}

// quotient of one element (bf16 value x) by the group scale, as compressed-tensors'
// `x / scale` (bf16 result; f32 for NVFP4).
__device__ __forceinline__ float qdiv(const QP& p, const GP& g, float x) {
  if (p.kind == K_NV) return x / g.s;
  return bfr(g.fast ? x * g.rs : x / g.s);
}

// encode: returns the code (int: q - qmin as unsigned; fp8: e4m3 byte; fp4: nibble)
__device__ __forceinline__ uint32_t encode(const QP& p, const GP& g, float x) {
  float t = qdiv(p, g, x);
  if (p.kind == K_INT) {
    if (!p.sym) t = bfr(t + g.zp);
    t = clamp_t(t, p.qmin, p.qmax);
    if (t != t) return (uint32_t)(-(int)p.qmin);  // round(NaN).to(int8) == 0 (D10)
    return __float_as_uint(t + p.magic) & ((1u << p.bits) - 1u);
  }
  if (p.kind == K_FP8) {
    t = clamp_t(t, -448.f, 448.f);
    return bf16_to_e4m3(f2bf(t));
  }
  t = clamp_t(t, -6.f, 6.f);
  return fp4_code(t);
}

// fake-quant of one int element straight from x: torch.round keeps the sign of zero, so a
// small negative quotient dequantizes to -0 (an int8 code cannot carry that sign)
__device__ __forceinline__ float fakequant_int(const QP& p, const GP& g, float x) {
  float t = qdiv(p, g, x);
  if (!p.sym) t = bfr(t + g.zp);
  t = clamp_t(t, p.qmin, p.qmax);
  return bfr(bfr(__builtin_rintf(t) - g.zp) * g.s);
}

// dequantize one code to the f32 value compressed-tensors' _dequantize produces before the
// final bf16 cast
__device__ __forceinline__ float decode(const QP& p, const GP& g, uint32_t code) {
  if (p.kind == K_INT) {
    float q = (float)((int)code + (int)p.qmin);
    return bfr(bfr(q - g.zp) * g.s);
  }
  if (p.kind == K_FP8) return bfr(e4m3_to_f32(code) * g.s);
  if (p.kind == K_NV) return bfr(fp4_value(code) * g.s);
  return bfr(fp4_value(code) * g.s);
}

// rebuild GP from stored qparams (qz_quantize_qparams / qz_dequantize)
__device__ __forceinline__ GP gp_from_stored(const QP& p, int scale_fmt, const void* scale,
                                              int64_t gi, const int8_t* zp, float gs) {
  GP g;
  g.zp = (zp && !p.sym) ? (float)zp[gi] : 0.f;
  if (p.kind == K_MX) {
    int byte = ((const uint8_t*)scale)[gi];
    g.sbits = byte;
    g.s = mx_pow2(byte - 127);
    g.rs = mx_pow2(127 - byte);
    g.fast = true;
    return g;
  }
  if (p.kind == K_NV) {
    uint32_t s8 = ((const uint8_t*)scale)[gi];
    g.sbits = s8;
    g.s = e4m3_to_f32(s8) / gs;
    g.rs = 0.f;
    g.fast = false;
    return g;
  }
  uint16_t sb = ((const uint16_t*)scale)[gi];
  g.sbits = sb;
  g.s = bf2f(sb);
  g.rs = __builtin_amdgcn_rcpf(g.s);
  g.fast = (g.s >= 0x1.0p-125f) && (g.s <= 0x1.0p+125f);
  return g;
}

// ------------------------------------------------ FP8_BLOCK single-pass path (qz_block.hip)
// n slices of a dense-row batch (tab == nullptr: slice b at w + b * ld_batch, codes / scales
// batch-major) or n table weights (tab: [4][n] {weight, codes, scales, 0}, qz_quantize_grouped)
struct BlockFp8Job {
  const void* w;
  int64_t n, rows, cols, ld_row, ld_batch;
  void* q_out;
  void* s_out;
  const uint64_t* tab;
};
bool block_fp8_ok(const BlockFp8Job& J);
int block_fp8_launch(const BlockFp8Job& J, const QP& p, hipStream_t st);

}  // namespace qz
