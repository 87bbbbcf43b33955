// qz_quant.hip -- weight quantize / pack kernels and their C-ABI entry points (gfx950).
//
// Two execution paths, identical results (both call qz_device.h's group_params/encode):
//  * the single-pass GROUP path (k_group_fast): contiguous bf16 weights, group_size = 8*2^k
//    (8..512).  Each lane owns 8 consecutive elements (one 16-B load); a wave-instruction
//    reads 1 KiB contiguous, so every load is fully coalesced whatever the row length; the
//    L = group_size/8 lanes of a group reduce min/max with xor-shuffles; each lane then
//    writes its 8 codes as one packed word (int4/fp4: 4 B, int8/fp8: 8 B) and the group's
//    first lane writes the scale.  HBM traffic = read once + write once.
//  * the generic path (k_minmax_generic -> k_qparams_keys -> k_quant_generic): any
//    strategy (tensor / channel / block / odd group sizes), strided or unaligned inputs, any
//    bit width; two reads of the weight.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "qz_device.h"

using namespace qz;

namespace {

constexpr int WAVE = 64;
constexpr int BLOCK = 256;
// 16-B units per lane per tile: 2 (round 1: 1 / 3 / 4 slower per weight launch; round 4
// re-check 23.72 / 24.00 / 20.24 us vs 20.04 us)
constexpr int UNROLL = 2;
// units per lane in the nt quantize path: 4 KiB tiles won (72.6 -> 69.3 us at [44032, 4096])
// only while the outputs stayed MALL-resident; with distinct outputs per weight UNROLL 2 / 3 / 4
// run 17.8 / 19.5 / 20.1 us per weight (grouped launches)
constexpr int UNROLL_NT = 2;
// tile size (units per lane) of a k_group_fast instantiation
constexpr int tile_unroll(bool fq, bool nt) { return (nt && !fq) ? UNROLL_NT : UNROLL; }
// threads per workgroup of the group path (one tile per wave); 64 / 256 measured equal / slower
constexpr int FBLOCK = 128;

// ------------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t pack2bf(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// float helpers for the generic path
template <int L>
__device__ __forceinline__ float grp_max(float v) {
#pragma unroll
  for (int m = 1; m < L; m <<= 1) v = fmaxf(v, __shfl_xor(v, m, WAVE));
  return v;
}
template <int L>
__device__ __forceinline__ float grp_min(float v) {
#pragma unroll
  for (int m = 1; m < L; m <<= 1) v = fminf(v, __shfl_xor(v, m, WAVE));
  return v;
}
constexpr int QZ_MAX_SEG = 8;  // shapes per mixed-shape grouped launch (qz_quantize_grouped_var)
struct FastArgs {
  const uint16_t* w;
  int64_t n_units;          // batch*rows*cols/8
  int64_t units_per_batch;  // rows*cols/8
  int64_t units_per_row;    // cols/8
  int64_t ld_batch;         // elements between batch slices (rows*cols when dense)
  QP p;
  int out_fmt;
  int scale_bytes;  // 2 (bf16) or 1 (e4m3 / e8m0)
  uint32_t wt_from;  // nt int4 path: workgroups from this linear id on store a lane quad's codes as one
                     // 16-B write-through store (wt_tail; 0xffffffff = never; every slice a multiple of 4 units)
  void* q_out;
  void* s_out;
  int8_t* zp_out;
  const float* gscale;      // [batch], NVFP4
  const float* col_scales;  // [cols] (+ b * cs_ld_batch), AWQ prescale (FQ only)
  int64_t cs_ld_batch;      // 0: one scale vector for every slice; cols: one per slice
  // grouped launch (qz_quantize_grouped): device table [4][n_tab] of per-weight pointers
  // {weight, codes, scale, zero point or 0}; blockIdx.y selects the weight.  Mixed shapes
  // (qz_quantize_grouped_var, n_seg > 0): the table holds runs of same-shape weights
  // ("segments"); segment i covers workgroups [seg_block[i], seg_block[i+1]) of a flat grid,
  // seg_bpw[i] workgroups per weight (divided by a host-computed magic: scalar ops only),
  // weights from seg_w0[i], seg_units[i] units each
  const uint64_t* tab;
  int64_t n_tab;
  int32_t n_seg;
  uint32_t seg_block[QZ_MAX_SEG + 1];
  uint32_t seg_bpw[QZ_MAX_SEG];
  uint32_t seg_magic[QZ_MAX_SEG];  // floor((2^32 - 1) / seg_bpw)
  uint32_t seg_w0[QZ_MAX_SEG];
  int64_t seg_units[QZ_MAX_SEG];
};

// --------------------------------------------------------------- single-pass path
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// fake-quant / tile path: weight bytes per launch above which loads are non-temporal (256 MiB)
constexpr int64_t QZ_NT_BYTES = 268435456;
// quantize (+pack): weight bytes per launch above which the group path streams non-temporally
// (nt loads + nt stores).  Measured with DISTINCT output tensors per weight, as a whole-model pass
// writes them (scripts/tune_fast.py OUTS=48 / MODE=grouped): the read-once weight must not take
// the MALL from the outputs, at every size -- int4 g128 [11008, 4096] per launch 21.4 -> 20.8 us,
// FP8 g32 25.3 -> 23.2 us, grouped launches 17.8 -> 17.3 us per weight (the sc1 stores measured
// better only while one shared output buffer stayed MALL-resident).
constexpr int64_t QZ_NT_BYTES_Q = 0;  // i.e. every quantize launch; its nt path stores non-temporally too
// per-weight launches stage through LDS-DMA (23.1 -> 21.5 us vs register loads), grouped launches
// load to registers (17.95 -> 17.51 us per weight): k_group_fast's REG = GRP
#ifndef QZ_BLK_FAST
#define QZ_BLK_FAST 1  // FP8_BLOCK 128x128 through qz_block.hip's strip kernel (0: the round-1 k_tile_fast)
#endif

// round both lanes of an f32 pair to bf16 and widen back: one v_cvt_pk_bf16_f32(0, v) per lane
// puts bf16(v) in the HIGH half over a zero low half -- the f32 value bf16(v) itself -- so 2 VALU
// per pair instead of a packed convert + 2 unpacks (3)
__device__ __forceinline__ f32x2 bfr2(f32x2 v) {
  f32x2 r;
  r.x = __uint_as_float(__builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){0.0f, v.x}, bf16x2)));
  r.y = __uint_as_float(__builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){0.0f, v.y}, bf16x2)));
  return r;
}

// bf16(d / c) for a bf16 value d and an f32 divisor c (AWQ's Q(W*s)/s): q = d * rcp(c) is
// within 2 ulps of the quotient, so bf16(q) is the answer unless q lies within 4 ulps of a bf16
// rounding midpoint (low 16 bits near 0x8000), where the IEEE division decides.
__device__ __forceinline__ float bf16_div(float d, float c) {
  const float q = d * __builtin_amdgcn_rcpf(c);
  const uint32_t b = __float_as_uint(q);
  if (__builtin_expect((((b & 0xffffu) + 4u - 0x8000u) & 0xffffu) < 8u || !(fabsf(c) >= 0x1.0p-100f && fabsf(c) <= 0x1.0p+100f), 0))
    return bfr(d / c);
  return bfr(q);
}

// Output stores outside the nt quantize path (the tile path, fake-quant, smoothing) are sc1
// (write-through): a plain store leaves the line dirty in the XCD's L2 and the end-of-kernel
// release writes it back in the kernel's tail (fake-quant [11008, 4096] 39.6 -> 37.3 us, smoothing
// 33.7 -> 31.1 us, FP8_BLOCK 25.4 -> 23.6 us; scripts/tune_ab.sh).  In the nt quantize path nt
// stores win once the outputs are distinct per weight (QZ_NT_BYTES_Q).  The 2-byte scale stores
// stay plain: as sc1 each is its own fabric write (no gain measured).
// sc1 store (relaxed agent-scope atomic store = global_store_* sc1)
template <typename T>
__device__ __forceinline__ void st_sc1(T* p, const T v) {
  if constexpr (sizeof(T) == 2) {
    __hip_atomic_store(reinterpret_cast<uint16_t*>(p), __builtin_bit_cast(uint16_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (sizeof(T) == 4) {
    __hip_atomic_store(reinterpret_cast<uint32_t*>(p), __builtin_bit_cast(uint32_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else if constexpr (sizeof(T) == 8) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), __builtin_bit_cast(uint64_t, v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  } else {
    *p = v;
  }
}

// output stores; NTS = non-temporal (streaming outputs of launches far larger than the MALL)
template <bool NTS, typename T>
__device__ __forceinline__ void st_out(T* p, const T v) {
  if constexpr (!NTS && sizeof(T) <= 8) {
    st_sc1(p, v);
  } else if constexpr (!NTS && sizeof(T) == 16) {
    st16_wt(p, __builtin_bit_cast(uint4, v));
  } else if constexpr (NTS) {
    if constexpr (sizeof(T) == 4) {
      __builtin_nontemporal_store(__builtin_bit_cast(uint32_t, v), reinterpret_cast<uint32_t*>(p));
    } else if constexpr (sizeof(T) == 8) {
      typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(__builtin_bit_cast(u32x2_t, v), reinterpret_cast<u32x2_t*>(p));
    } else {
      __builtin_nontemporal_store(__builtin_bit_cast(u32x4, v), reinterpret_cast<u32x4*>(p));
    }
  } else {
    *p = v;
  }
}

// two f32 -> packed bf16 pair (one v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
// packed bf16(d / c) for a pair: bf16_div's rcp path on both lanes, the IEEE division for a
// pair with a quotient near a bf16 midpoint
__device__ __forceinline__ uint32_t bf16_div_pk(f32x2 d, f32x2 c) {
  const f32x2 r = {__builtin_amdgcn_rcpf(c.x), __builtin_amdgcn_rcpf(c.y)};
  const f32x2 q = d * r;
  const uint32_t bx = __float_as_uint(q.x), by = __float_as_uint(q.y);
  const bool near = ((((bx & 0xffffu) + 4u - 0x8000u) & 0xffffu) < 8u) | ((((by & 0xffffu) + 4u - 0x8000u) & 0xffffu) < 8u);
  const bool range = (fabsf(c.x) >= 0x1.0p-100f) & (fabsf(c.x) <= 0x1.0p+100f) & (fabsf(c.y) >= 0x1.0p-100f) &
                     (fabsf(c.y) <= 0x1.0p+100f);
  if (__builtin_expect(near || !range, 0)) return pk_bf16(f32x2{d.x / c.x, d.y / c.y});
  return pk_bf16(q);
}

// NVFP4 quotient x / s clamped to the E2M1 range, "+ 0" turning -0 into +0 (torch.sign(-0.) is
// 0); a NaN quotient (0 / 0: a zero element of a slice whose global scale overflowed to inf)
// encodes as code 0 whatever its sign bit (D17)
__device__ __forceinline__ float nv_clamp(float q) {
  return q != q ? 0.0f : __builtin_amdgcn_fmed3f(q, -6.f, 6.f) + 0.0f;
}

// quotient, round/clamp/encode and store of one 8-element unit whose group params are known.
// unit = dense output unit index.  Returns false for invalid (out-of-range) units.
template <int KIND, bool FQ, bool SYM, bool NTS = false>
__device__ __forceinline__ void encode_store(const FastArgs& A, const QP& p, const GP& g, const f32x2* x,
                                             const f32x2* cs, const int64_t unit) {

  // ---- NVFP4, quantize only: the f32 quotient x / s is decided from q = x * rcp(s), which is
  // within 3 ulps of it.  The E2M1 rounding boundaries (0.25 0.75 1.25 1.75 2.5 3.5 5) have
  // only their top 2 mantissa bits set, so q can round differently from x / s only if its low
  // 21 mantissa bits are within 4 of zero (mod 2^21); such pairs (and +-0, which needs the
  // signed-zero rule) take the IEEE division.  Exact grid values may be flagged too (harmless).
  if (KIND == K_NV && !FQ) {
    // near: the low 21 bits of (bits + 4) below 8, i.e. ((bits << 11) + (4 << 11)) < (8 << 11)
    // (one v_lshl_add_u32 each), either element of the pair (v_min_u32); each pair's two codes
    // go straight into byte k of the word (the conversion's destination-byte select)
    float ca[4], cb[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float qa = x[k].x * g.rs, qb = x[k].y * g.rs;
      const bool near = min((__float_as_uint(qa) << 11) + 0x2000u, (__float_as_uint(qb) << 11) + 0x2000u) < 0x4000u;
      if (__builtin_expect(near || !g.fast, 0)) {
        ca[k] = nv_clamp(x[k].x / g.s);
        cb[k] = nv_clamp(x[k].y / g.s);
      } else {
        ca[k] = __builtin_amdgcn_fmed3f(qa, -6.f, 6.f);
        cb[k] = __builtin_amdgcn_fmed3f(qb, -6.f, 6.f);
      }
    }
    uint32_t word = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, ca[0], cb[0], 1.0f, 0);
    word = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(word, ca[1], cb[1], 1.0f, 1);
    word = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(word, ca[2], cb[2], 1.0f, 2);
    word = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(word, ca[3], cb[3], 1.0f, 3);
    st_out<NTS>(reinterpret_cast<uint32_t*>(A.q_out) + unit, word);
    return;
  }

  // ---- quotient x / scale (bf16; f32 for NVFP4); x * rcp(s) is exact-equivalent (rcp lemma)
  f32x2 t[4];
  if (KIND == K_NV) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { t[k].x = x[k].x / g.s; t[k].y = x[k].y / g.s; }
  } else {
    const f32x2 rs2 = {g.rs, g.rs};
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = x[k] * rs2;
    if (__builtin_expect(!g.fast, 0)) {
#pragma unroll
      for (int k = 0; k < 4; ++k) { t[k].x = x[k].x / g.s; t[k].y = x[k].y / g.s; }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) t[k] = bfr2(t[k]);
  }

  if (KIND == K_INT) {
    // clamp (bf16 bounds), then t + (2^23 - qmin): RNE(t) - qmin lands in the low mantissa bits
    f32x2 q[4];
    const f32x2 mg = {p.magic, p.magic};
    const f32x2 zp2 = {g.zp, g.zp};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x2 tk = t[k];
      if (!SYM) tk = bfr2(tk + zp2);
      tk.x = __builtin_amdgcn_fmed3f(tk.x, p.qmin, p.qmax);
      tk.y = __builtin_amdgcn_fmed3f(tk.y, p.qmin, p.qmax);
      t[k] = tk;
      q[k] = tk + mg;
    }
    if (FQ) {
      // pairwise: bf16(bf16(round(t) - zp) * s) [/ col scale], the last bf16 rounding packs the
      // output word directly (round() keeps the sign of zero: -0 dequantizes to -0)
      const f32x2 s2 = {g.s, g.s};
      uint32_t o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x2 r = {__builtin_rintf(t[k].x), __builtin_rintf(t[k].y)};
        const f32x2 dq = bfr2(bfr2(r - zp2) * s2);
        o[k] = A.col_scales ? bf16_div_pk(dq, cs[k]) : pk_bf16(dq);
      }
      st_out<NTS>(reinterpret_cast<uint4*>(A.q_out) + unit, make_uint4(o[0], o[1], o[2], o[3]));
    } else if (A.out_fmt == QZ_OUT_PACKED_INT32 && p.bits == 4) {
      // the low byte of each float 0x4B0000uu is its code u (< 16): gather the even elements'
      // bytes into E and the odd ones' into O (v_perm_b32), word = E | O << 4 (7 VALU for 8 codes)
      const uint32_t e_lo = __builtin_amdgcn_perm(__float_as_uint(q[1].x), __float_as_uint(q[0].x), 0x0c0c0400u);
      const uint32_t e_hi = __builtin_amdgcn_perm(__float_as_uint(q[3].x), __float_as_uint(q[2].x), 0x04000c0cu);
      const uint32_t o_lo = __builtin_amdgcn_perm(__float_as_uint(q[1].y), __float_as_uint(q[0].y), 0x0c0c0400u);
      const uint32_t o_hi = __builtin_amdgcn_perm(__float_as_uint(q[3].y), __float_as_uint(q[2].y), 0x04000c0cu);
      const uint32_t word = ((o_lo | o_hi) << 4) | (e_lo | e_hi);
      if (NTS && wt_tail(A.wt_from) && (reinterpret_cast<uintptr_t>(A.q_out) & 15u) == 0) {
        // the 4 words of a lane quad (4 consecutive units of one slice: 16 contiguous bytes; the
        // host sets wt only when every slice holds a multiple of 4 units, so a quad is valid as a
        // whole) gathered into its first lane by DPP quad broadcasts, one 16-B write-through store;
        // a codes buffer that is not 16-B aligned (a caller's table entry) keeps the 4-B stores
        const uint32_t w1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)word, 0x55, 0xF, 0xF, true);
        const uint32_t w2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)word, 0xAA, 0xF, 0xF, true);
        const uint32_t w3 = (uint32_t)__builtin_amdgcn_mov_dpp((int)word, 0xFF, 0xF, 0xF, true);
        if ((__lane_id() & 3) == 0) st16_wt(reinterpret_cast<uint32_t*>(A.q_out) + unit, make_uint4(word, w1, w2, w3));
      } else {
        st_out<NTS>(reinterpret_cast<uint32_t*>(A.q_out) + unit, word);
      }
    } else {
      uint32_t c[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        c[2 * k] = __float_as_uint(q[k].x) & 0xffu;
        c[2 * k + 1] = __float_as_uint(q[k].y) & 0xffu;
      }
      if (A.out_fmt == QZ_OUT_PACKED_INT32) {  // 8 bits: u = q + 128, 4 per word
        st_out<NTS>(reinterpret_cast<uint2*>(A.q_out) + unit, make_uint2(c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24),
                                                             c[4] | (c[5] << 8) | (c[6] << 16) | (c[7] << 24)));
      } else {  // int8 (signed) bytes
        const uint32_t off = (uint32_t)(-(int)p.qmin);
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = (c[i] - off) & 0xffu;
        st_out<NTS>(reinterpret_cast<uint2*>(A.q_out) + unit, make_uint2(c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24),
                                                             c[4] | (c[5] << 8) | (c[6] << 16) | (c[7] << 24)));
      }
    }
  } else {
    uint32_t c[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (KIND == K_FP8) {
        // v_cvt_pk_fp8_f32 (OCP e4m3, RNE); exhaustively checked vs torch's cast
        const uint32_t pk = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(t[k].x, -448.f, 448.f),
                                                                      __builtin_amdgcn_fmed3f(t[k].y, -448.f, 448.f), 0, false);
        c[2 * k] = pk & 0xffu;
        c[2 * k + 1] = (pk >> 8) & 0xffu;
      } else {
        // v_cvt_scalef32_pk_fp4_f32: RNE on the E2M1 grid == cast_to_fp4's thresholds (checked
        // exhaustively); "+ 0" maps an exact -0 input to +0 (torch.sign(-0.) is 0 -> code 0),
        // small negatives still round to -0 (code 8) as sign(x)*|q| does
        const float ca = KIND == K_NV ? nv_clamp(t[k].x) : __builtin_amdgcn_fmed3f(t[k].x, -6.f, 6.f) + 0.0f;
        const float cb = KIND == K_NV ? nv_clamp(t[k].y) : __builtin_amdgcn_fmed3f(t[k].y, -6.f, 6.f) + 0.0f;
        const uint32_t pk = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(0u, ca, cb, 1.0f, 0);
        c[2 * k] = pk & 0xfu;
        c[2 * k + 1] = (pk >> 4) & 0xfu;
      }
    }
    if (FQ) {
      float d[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        d[i] = decode(p, g, c[i]);
        if (A.col_scales) d[i] = bf16_div(d[i], (i & 1) ? cs[i >> 1].y : cs[i >> 1].x);
      }
      uint4 o = make_uint4(pack2bf(d[0], d[1]), pack2bf(d[2], d[3]), pack2bf(d[4], d[5]), pack2bf(d[6], d[7]));
      st_out<NTS>(reinterpret_cast<uint4*>(A.q_out) + unit, o);
    } else if (KIND == K_FP8) {
      st_out<NTS>(reinterpret_cast<uint2*>(A.q_out) + unit, make_uint2(c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24),
                                                           c[4] | (c[5] << 8) | (c[6] << 16) | (c[7] << 24)));
    } else {  // fp4 packed: element 2k in the low nibble of byte k
      uint32_t word = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) word |= c[i] << (4 * i);
      st_out<NTS>(reinterpret_cast<uint32_t*>(A.q_out) + unit, word);
    }
  }
}

// Process one 8-element unit: observe (group reduce over L lanes), qparams, quantize, store.
template <int LOGL, int KIND, bool FQ, bool SYM, bool NTS = false>
__device__ __forceinline__ void process_unit(const FastArgs& A, const QP& p, const uint4 v, const int64_t unit,
                                             const bool valid, const float gs, const int lane, const int64_t b,
                                             const f32x2* cs_in) {
  constexpr int L = 1 << LOGL;
  // unit: dense output index (batch*units_per_batch + local); valid is uniform within a group
  const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
  f32x2 x[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    x[k].x = __uint_as_float(wd[k] << 16);
    x[k].y = __uint_as_float(wd[k] & 0xffff0000u);
  }
  f32x2 cs[4];
  if (FQ && A.col_scales) {  // column scales were fetched with the tile (k_group_fast)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      cs[k] = cs_in[k];
      x[k] = bfr2(x[k] * cs[k]);  // W * s in the weight dtype
    }
  }

  // ---- observe: memoryless min/max over the group (exact in bf16), on integer keys
  float mn, mx;
  if (SYM) {
    uint32_t am;
    if (FQ && A.col_scales) {
      am = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        am = max(am, max(__float_as_uint(x[k].x) & 0x7fffffffu, __float_as_uint(x[k].y) & 0x7fffffffu));
    } else {  // |bf16| bit patterns, two per dword: v_pk_max_u16 on the raw words
      const uint32_t m = pk_max_u16(pk_max_u16(wd[0] & 0x7fff7fffu, wd[1] & 0x7fff7fffu),
                                    pk_max_u16(wd[2] & 0x7fff7fffu, wd[3] & 0x7fff7fffu));
      am = max(m & 0xffffu, m >> 16) << 16;
    }
    am = grp_max_u<L>(am);
    mx = __uint_as_float(am);
    mn = -mx;
  } else {
    uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a = f2key(x[k].x), b = f2key(x[k].y);
      kmn = min(kmn, min(a, b));
      kmx = max(kmx, max(a, b));
    }
    mn = key2f(grp_min_u<L>(kmn));
    mx = key2f(grp_max_u<L>(kmx));
  }
  QP ps = p;
  ps.sym = SYM;
  // symmetric: mx is the group's absmax
  const GP g = (SYM && (KIND == K_INT || KIND == K_FP8 || KIND == K_FP4)) ? group_params_sym(ps, mx)
                                                                          : group_params(ps, mn, mx, gs, SYM);
  if (!valid) return;
  encode_store<KIND, FQ, SYM, NTS>(A, ps, g, x, cs, unit);
  if ((lane & (L - 1)) == 0) {
    const int64_t gi = unit >> LOGL;
    if (A.scale_bytes == 2) {
      reinterpret_cast<uint16_t*>(A.s_out)[gi] = (uint16_t)g.sbits;
    } else {
      reinterpret_cast<uint8_t*>(A.s_out)[gi] = (uint8_t)g.sbits;
    }
    if (A.zp_out) A.zp_out[gi] = (int8_t)g.zp;
  }
}

template <int LOGL, int KIND, bool FQ, bool SYM, bool NTS, int UNROLL>
__device__ __forceinline__ void process_tile(const FastArgs& A, const QP& p, const uint4* v, int64_t b, int64_t tile,
                                             int lane, const f32x2 (*csu)[4]) {
  const float gs = (KIND == K_NV) ? A.gscale[b] : 0.f;
#pragma unroll
  for (int u = 0; u < UNROLL; ++u) {
    const int64_t local = tile * (UNROLL * WAVE) + u * WAVE + lane;
    const int64_t unit = b * A.units_per_batch + local;
    const bool valid = local < A.units_per_batch;
    process_unit<LOGL, KIND, FQ, SYM, NTS>(A, p, v[u], unit, valid, gs, lane, b, csu[u]);
  }
}

// One tile (UNROLL*64 units = UNROLL KiB of bf16) per wave.  The tile is streamed HBM -> LDS
// with global_load_lds_dwordx4 (LDS-DMA: no VGPR destination, 1 KiB per wave-instruction,
// fully coalesced), the wave waits on its own vmcnt and reads its lanes' 16 B back with
// ds_read_b128; latency is hidden by occupancy (one-shot waves, up to 8 per SIMD).  Measured on
// MI355X (scripts/tune_fast.py): LDS-DMA staging is 5 % faster than register loads here, and a
// persistent grid-stride loop with register double-buffering is slower than one-shot waves.
// Out-of-range lanes re-load the slice's last unit (results never stored), keeping the
// loads branch-free.  grid = (tiles per slice, batch): slices may be strided (fused experts).
template <int LOGL, int KIND, bool FQ, bool SYM, bool NT = false, bool GRP = false>
__global__ __launch_bounds__(FBLOCK) void k_group_fast(FastArgs A0) {
  constexpr int UNROLL = tile_unroll(FQ, NT);
  __shared__ uint4 lds_buf[FBLOCK / WAVE][UNROLL][WAVE];
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x >> 6;
  FastArgs A = A0;
  int64_t b = blockIdx.y;
  int64_t blk = blockIdx.x;
  if constexpr (GRP) {
    if (A0.n_seg > 0) {  // mixed shapes: segment, weight and local workgroup (uniform, SALU)
      const uint32_t x = (uint32_t)blk;
      int sg = 0;
#pragma unroll
      for (int i = 1; i < QZ_MAX_SEG; ++i) sg += (i < A0.n_seg) & (x >= A0.seg_block[i]);
      const uint32_t rel = x - A0.seg_block[sg], d = A0.seg_bpw[sg];
      uint32_t q = __umulhi(rel, A0.seg_magic[sg]);  // floor(rel / d) or one less
      uint32_t r = rel - q * d;
      if (r >= d) { ++q; r -= d; }
      b = A0.seg_w0[sg] + q;
      blk = r;
      A.units_per_batch = A0.seg_units[sg];
    }
  }
  const int64_t tile = blk * (FBLOCK / WAVE) + w;
  const int64_t tiles = (A.units_per_batch + UNROLL * WAVE - 1) / (UNROLL * WAVE);
  if (tile >= tiles) return;
  if constexpr (GRP) {  // grouped launch: this workgroup's weight and outputs from the table
    // table entries are global-memory pointers; casting through address space 1 makes the
    // compiler emit global_* instead of flat_* loads and stores, which measured SLOWER here
    // (grouped int4 g128, 100 weights: 17.09 -> 18.16 us/weight, r02g A/B), so flat it stays
    A.w = reinterpret_cast<const uint16_t*>(A0.tab[b]);
    A.q_out = reinterpret_cast<void*>(A0.tab[A0.n_tab + b]);
    A.s_out = reinterpret_cast<void*>(A0.tab[2 * A0.n_tab + b]);
    A.zp_out = reinterpret_cast<int8_t*>(A0.tab[3 * A0.n_tab + b]);
    b = 0;
  }
  const uint4* src = reinterpret_cast<const uint4*>(A.w + b * A.ld_batch);
  // direct-to-register 16-B loads (grouped launches) or LDS-DMA staging (per-weight launches)
  constexpr bool REG = GRP;
  uint4 v[UNROLL];
  if constexpr (REG) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t unit = tile * (UNROLL * WAVE) + u * WAVE + lane;
      unit = unit < A.units_per_batch ? unit : A.units_per_batch - 1;
      if constexpr (NT) v[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + unit)));
      else v[u] = src[unit];
    }
  } else {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t unit = tile * (UNROLL * WAVE) + u * WAVE + lane;
      unit = unit < A.units_per_batch ? unit : A.units_per_batch - 1;
      __builtin_amdgcn_global_load_lds((const void*)(src + unit),
                                       (__attribute__((address_space(3))) void*)&lds_buf[w][u][0], 16, 0,
                                       NT ? 2 : 0);
    }
  }
  // AWQ fake-quant: fetch this lane's column scales while the DMA is in flight
  f32x2 csu[UNROLL][4];
  if (FQ && A.col_scales) {
    const float* cs_b = A.col_scales + b * A.cs_ld_batch;
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      int64_t unit = tile * (UNROLL * WAVE) + u * WAVE + lane;
      unit = unit < A.units_per_batch ? unit : A.units_per_batch - 1;
      const int64_t c0 = (A.units_per_batch < (int64_t)1 << 32 ? (int64_t)((uint32_t)unit % (uint32_t)A.units_per_row)
                                                                  : unit % A.units_per_row) * 8;
      const float4 c_lo = *reinterpret_cast<const float4*>(cs_b + c0);
      const float4 c_hi = *reinterpret_cast<const float4*>(cs_b + c0 + 4);
      csu[u][0] = f32x2{c_lo.x, c_lo.y}; csu[u][1] = f32x2{c_lo.z, c_lo.w};
      csu[u][2] = f32x2{c_hi.x, c_hi.y}; csu[u][3] = f32x2{c_hi.z, c_hi.w};
    }
  }
  QP p = A.p;
  p.kind = KIND;
  if constexpr (!REG) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA has landed in LDS
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = lds_buf[w][u][lane];
  }
  process_tile<LOGL, KIND, FQ, SYM, NT, UNROLL>(A, p, v, b, tile, lane, csu);
}

// ------------------------------------------------ AWQ fake-quant with column scales
// Q(W*s)/s of the AWQ grid (qz_awq_fake_quant[_batched]; group strategy, power-of-two groups of
// 8..512, dense rows).  A wave's tile is FQ_ROWS rows x 64 lanes, and every lane owns the SAME 8
// columns in each of those rows, so the column scales, their reciprocals and the range check
// are fetched / computed once per tile instead of once per 8 elements.  The unit-wise
// k_group_fast<..., FQ=true> issued 457 VALU instructions per wave (2 units per lane) and was
// VALU-bound (PMC r02c: 41.9 us for [11008, 4096], 0.54 of 8 TB/s).  grid = (column chunks of
// 64 units, row blocks / waves per workgroup, batch): consecutive workgroups cover one row
// block's chunks, so the stream stays contiguous.
constexpr int FQ_ROWS = 4;  // rows per tile: 2 / 4 / 8 = 31.93 / 30.37 / 33.25 us (r02e)

// bf16(d / c) for a pair given r = rcp(c), packed: the IEEE division only when a quotient lies
// within 4 ulps of a bf16 rounding midpoint (low 16 bits near 0x8000; 16-bit adds) or when
// the lane's column scales are outside the range where rcp is accurate (ok == false)
// near-midpoint test of a quotient pair: the two low halves packed (v_perm), +0x8004 on both
// (v_pk_add_u16), then the smaller half below 8 means one of them is within 4 ulps of 0x8000
__device__ __forceinline__ bool near_mid_pk(const f32x2 q) {
  const uint32_t lo = __builtin_amdgcn_perm(__float_as_uint(q.y), __float_as_uint(q.x), 0x05040100u);
  const u16x2 a = __builtin_bit_cast(u16x2, lo) + (u16x2){0x8004, 0x8004};
  return min(a.x, a.y) < 8;
}

// widen a packed bf16 pair to f32
__device__ __forceinline__ f32x2 unpk(const uint32_t u) {
  return f32x2{__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u)};
}

// one unit (8 elements of one row, one lane): W' = bf16(W * s) -> observe the group of W' ->
// qparams -> quantize -> dequantize -> bf16(fl32(dq / s)); the same op sequence as
// encode_store<KIND, FQ=true> (compressed-tensors' fake_quantize on the scaled weight, then the
// f32 division by the column scales)
template <int LOGL, int KIND, bool SYM>
__device__ __forceinline__ uint4 fq_unit(const QP& p, const uint4 v, const f32x2* cs, const f32x2* rc, const bool cs_ok) {
  constexpr int L = 1 << LOGL;
  const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
  f32x2 x[4];
  float mn, mx;
  // W * s rounded to bf16 straight into f32 lanes (bfr2: one convert per element) and the
  // group's |max| by three-input maxima with |.| source modifiers (4 VALU for 8 elements);
  // the inputs are finite (D12), so the maximum is exact and order-free
  if (SYM) {
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = bfr2(unpk(wd[k]) * cs[k]);
    float m0, m1, m2, m3;
    asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(m0) : "v"(x[0].x), "v"(x[0].y), "v"(x[1].x));
    asm("v_max3_f32 %0, |%1|, |%2|, |%3|" : "=v"(m1) : "v"(x[1].y), "v"(x[2].x), "v"(x[2].y));
    asm("v_max3_f32 %0, %1, %2, |%3|" : "=v"(m2) : "v"(m0), "v"(m1), "v"(x[3].x));
    asm("v_max_f32 %0, %1, |%2|" : "=v"(m3) : "v"(m2), "v"(x[3].y));
    mx = __uint_as_float(grp_max_u<L>(__float_as_uint(m3)));
    mn = -mx;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = bfr2(unpk(wd[k]) * cs[k]);  // W * s in the weight dtype
    uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t a = f2key(x[k].x), b = f2key(x[k].y);
      kmn = min(kmn, min(a, b));
      kmx = max(kmx, max(a, b));
    }
    mn = key2f(grp_min_u<L>(kmn));
    mx = key2f(grp_max_u<L>(kmx));
  }
  QP ps = p;
  ps.sym = SYM;
  ps.kind = KIND;
  const GP g = (SYM && KIND != K_MX) ? group_params_sym(ps, mx) : group_params(ps, mn, mx, 0.f, SYM);
  // quotient x / scale in bf16 (x * rcp(s): rcp lemma)
  f32x2 t[4];
  const f32x2 rs2 = {g.rs, g.rs};
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = x[k] * rs2;
  if (__builtin_expect(!g.fast, 0)) {
#pragma unroll
    for (int k = 0; k < 4; ++k) { t[k].x = x[k].x / g.s; t[k].y = x[k].y / g.s; }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) t[k] = bfr2(t[k]);
  const f32x2 s2 = {g.s, g.s};
  f32x2 dq[4];
  if (KIND == K_INT) {
    const f32x2 zp2 = {g.zp, g.zp};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x2 tk = t[k];
      if (!SYM) tk = bfr2(tk + zp2);
      const f32x2 r = {__builtin_rintf(__builtin_amdgcn_fmed3f(tk.x, p.qmin, p.qmax)),
                       __builtin_rintf(__builtin_amdgcn_fmed3f(tk.y, p.qmin, p.qmax))};
      // symmetric: the zero point is 0 and r - 0 == r exactly (sign of zero kept)
      dq[k] = SYM ? bfr2(r * s2) : bfr2(bfr2(r - zp2) * s2);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint32_t c0, c1;
      if (KIND == K_FP8) {
        const uint32_t pk = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(t[k].x, -448.f, 448.f),
                                                                      __builtin_amdgcn_fmed3f(t[k].y, -448.f, 448.f), 0, false);
        c0 = pk & 0xffu;
        c1 = (pk >> 8) & 0xffu;
      } else {  // MXFP4 / FP4 (E2M1 RNE, as encode_store)
        const uint32_t pk = __builtin_amdgcn_cvt_scalef32_pk_fp4_f32(
            0u, __builtin_amdgcn_fmed3f(t[k].x, -6.f, 6.f) + 0.0f, __builtin_amdgcn_fmed3f(t[k].y, -6.f, 6.f) + 0.0f,
            1.0f, 0);
        c0 = pk & 0xfu;
        c1 = (pk >> 4) & 0xfu;
      }
      dq[k] = f32x2{decode(ps, g, c0), decode(ps, g, c1)};
    }
  }
  // ÷ column scale: bf16(d * rcp(c)) unless a quotient is within 4 ulps of a bf16 rounding
  // midpoint or a scale is outside rcp's accurate range -- then the IEEE division (one branch
  // per unit; taken by ~6 % of the waves' units on Gaussian weights)
  f32x2 q[4];
  bool near = !cs_ok;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    q[k] = dq[k] * rc[k];
    near |= near_mid_pk(q[k]);
  }
  if (__builtin_expect(near, 0)) {
#pragma unroll
    for (int k = 0; k < 4; ++k) q[k] = f32x2{dq[k].x / cs[k].x, dq[k].y / cs[k].y};
  }
  return make_uint4(pk_bf16(q[0]), pk_bf16(q[1]), pk_bf16(q[2]), pk_bf16(q[3]));
}

// one tile per wave (several consecutive tiles per wave, the next one's loads in flight,
// measured slower: profiles/r02ay_fq_tiles_ab.log)

template <bool NT, int U>
__device__ __forceinline__ void fq_load_tile(uint4 (&v)[U], const uint4* src, int64_t r0, int64_t rows, int64_t upr,
                                             int64_t cuc) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    int64_t r = r0 + u;
    r = r < rows ? r : rows - 1;
    const uint4* ptr = src + r * upr + cuc;
    if constexpr (NT) v[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(ptr)));
    else v[u] = *ptr;
  }
}

// buffer stores sc1 (gfx950 CPol SC1 = 16), weight loads default policy: nt loads / stores and
// plain stores measured equal or slower in the AWQ grid's pattern (r04v / r04ad)
constexpr int FQ_ST_AUX = 16, FQ_LD_AUX = 0;
// wave-uniform 64-bit value, provably so to the compiler (SGPRs)
__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)v) |
         ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32);
}

template <int LOGL, int KIND, bool SYM, bool NT>
__global__ __launch_bounds__(FBLOCK) void k_fq_cols(FastArgs A, int64_t rows) {
  constexpr int U = FQ_ROWS;
  const int lane = threadIdx.x & (WAVE - 1);
  // this wave's tile (wave index through readfirstlane: wave-uniform to the compiler)
  const int64_t rblk = (int64_t)blockIdx.y * (FBLOCK / WAVE) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (rblk * U >= rows) return;
  const int64_t b = blockIdx.z;
  const int64_t upr = A.units_per_row;
  const int64_t cu = (int64_t)blockIdx.x * WAVE + lane;  // this lane's column unit
  const bool col_ok = cu < upr;
  const int64_t cuc = col_ok ? cu : upr - 1;
  const uint4* src = reinterpret_cast<const uint4*>(A.w + b * A.ld_batch);
  uint4 v[U];
  // one tile per wave: the tile's rows through one source and one destination descriptor
  // (wave-uniform bases, 32-bit lane / row offsets: no per-unit 64-bit address arithmetic); rows
  // past the slice re-read its last row and are not stored, nor are lanes past the last column
  constexpr bool BUF = !NT;  // wave-uniform buffer descriptors (the nt variant uses global loads)
  uint32_t voff = 0, roff[U];
  __amdgpu_buffer_rsrc_t rs_dst;
  int nrow_b = 0;
  if constexpr (BUF) {
    const int64_t r0 = rblk * U;
    nrow_b = (int)min<int64_t>(U, rows - r0);
    const uint32_t rowb = (uint32_t)upr * 16u;
    voff = (uint32_t)cuc * 16u;
#pragma unroll
    for (int u = 0; u < U; ++u) roff[u] = __builtin_amdgcn_readfirstlane((uint32_t)min(u, nrow_b - 1) * rowb);
    const auto rs_src = __builtin_amdgcn_make_buffer_rsrc((void*)uni64((uint64_t)(src + r0 * upr)), 0, 0x7fffffff,
                                                          0x00020000);
    rs_dst = __builtin_amdgcn_make_buffer_rsrc(
        (void*)uni64((uint64_t)(reinterpret_cast<uint4*>(A.q_out) + b * A.units_per_batch + r0 * upr)), 0, 0x7fffffff,
        0x00020000);
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs_src, voff, roff[u], FQ_LD_AUX));
  } else {
    fq_load_tile<NT, U>(v, src, rblk * U, rows, upr, cuc);
  }
  // this lane's 8 column scales, their reciprocals, and whether rcp is accurate for all 8
  const float* csp = A.col_scales + b * A.cs_ld_batch + cuc * 8;
  const float4 c_lo = *reinterpret_cast<const float4*>(csp);
  const float4 c_hi = *reinterpret_cast<const float4*>(csp + 4);
  const f32x2 cs[4] = {{c_lo.x, c_lo.y}, {c_lo.z, c_lo.w}, {c_hi.x, c_hi.y}, {c_hi.z, c_hi.w}};
  f32x2 rc[4];
  bool cs_ok = true;  // false for a zero / tiny / huge / non-finite scale (comparisons fail on NaN)
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    rc[k] = f32x2{__builtin_amdgcn_rcpf(cs[k].x), __builtin_amdgcn_rcpf(cs[k].y)};
    cs_ok &= (fabsf(cs[k].x) >= 0x1.0p-100f) & (fabsf(cs[k].x) <= 0x1.0p+100f) & (fabsf(cs[k].y) >= 0x1.0p-100f) &
             (fabsf(cs[k].y) <= 0x1.0p+100f);
  }
  const QP p = A.p;
  if constexpr (BUF) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4 o = fq_unit<LOGL, KIND, SYM>(p, v[u], cs, rc, cs_ok);
      if (col_ok && u < nrow_b)  // sc1 (write-through) as st_out
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs_dst, voff, roff[u], FQ_ST_AUX);
    }
    return;
  }
  const int64_t r0 = rblk * U;
  uint4* dst = reinterpret_cast<uint4*>(A.q_out) + b * A.units_per_batch + r0 * upr + cuc;
  const int nrow = (int)min<int64_t>(U, rows - r0);  // rows of this tile inside the slice
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint4 o = fq_unit<LOGL, KIND, SYM>(p, v[u], cs, rc, cs_ok);
    if (col_ok && u < nrow) st_out<false>(dst, o);
    dst += upr;
  }
}

// --------------------------------------------------------------- single-pass tile path
// One workgroup per quantization group that is too large (or too 2-D) for a lane group: a
// BLOCK tile (e.g. FP8_BLOCK 128x128), a CHANNEL row, or a group wider than 512.  The tile
// (<= 256 threads x MAXU units of 8 bf16) is held in registers, min/max reduce across the
// workgroup (DPP within the wave, LDS across the 4 waves), then every unit is encoded from
// registers: one HBM read, like the group path.
struct TileArgs {
  int64_t rows, tile_rows, tile_w8, tiles_c, ld_row;  // tile_w8 = tile width in units
};

template <int KIND, bool SYM, int MAXU, bool NT = false>
__global__ __launch_bounds__(BLOCK) void k_tile_fast(FastArgs A, TileArgs T) {
  __shared__ uint32_t red[2][BLOCK / WAVE];
  const int64_t b = blockIdx.y;
  const int64_t tid = blockIdx.x;
  const int64_t tr = tid / T.tiles_c, tc = tid % T.tiles_c;
  const uint32_t U = (uint32_t)(T.tile_rows * T.tile_w8);
  const uint16_t* wb = A.w + b * A.ld_batch;
  uint4 v[MAXU];
  int64_t oidx[MAXU];
#pragma unroll
  for (int i = 0; i < MAXU; ++i) {
    const uint32_t u = threadIdx.x + i * BLOCK;
    const uint32_t uu = u < U ? u : U - 1;
    const int64_t row = tr * T.tile_rows + uu / (uint32_t)T.tile_w8;
    const int64_t c8 = tc * T.tile_w8 + uu % (uint32_t)T.tile_w8;
    const u32x4* src = reinterpret_cast<const u32x4*>(wb + row * T.ld_row + c8 * 8);
    const u32x4 t = NT ? __builtin_nontemporal_load(src) : *src;
    v[i] = make_uint4(t.x, t.y, t.z, t.w);
    oidx[i] = (u < U) ? (b * T.rows + row) * A.units_per_row + c8 : -1;
  }
  QP p = A.p;
  p.kind = KIND;
  p.sym = SYM;
  // per-thread then workgroup min/max on integer keys
  uint32_t kmn = 0xffffffffu, kmx = 0u;
#pragma unroll
  for (int i = 0; i < MAXU; ++i) {
    if (oidx[i] < 0) continue;
    const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float lo = __uint_as_float(wd[k] << 16), hi = __uint_as_float(wd[k] & 0xffff0000u);
      if (SYM) {
        kmx = max(kmx, max(__float_as_uint(lo) & 0x7fffffffu, __float_as_uint(hi) & 0x7fffffffu));
      } else {
        const uint32_t ka = f2key(lo), kb = f2key(hi);
        kmn = min(kmn, min(ka, kb));
        kmx = max(kmx, max(ka, kb));
      }
    }
  }
  kmx = grp_max_u<WAVE>(kmx);
  if (!SYM) kmn = grp_min_u<WAVE>(kmn);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = kmn; red[1][w] = kmx; }
  __syncthreads();
  kmn = red[0][0];
  kmx = red[1][0];
#pragma unroll
  for (int k = 1; k < BLOCK / WAVE; ++k) { kmn = min(kmn, red[0][k]); kmx = max(kmx, red[1][k]); }
  float mn, mx;
  if (SYM) { mx = __uint_as_float(kmx); mn = -mx; }
  else { mn = key2f(kmn); mx = key2f(kmx); }
  const GP g = group_params(p, mn, mx, 0.f);
  f32x2 cs[4];
#pragma unroll
  for (int i = 0; i < MAXU; ++i) {
    if (oidx[i] < 0) continue;
    const uint32_t wd[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
    f32x2 x[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { x[k].x = __uint_as_float(wd[k] << 16); x[k].y = __uint_as_float(wd[k] & 0xffff0000u); }
    encode_store<KIND, false, SYM>(A, p, g, x, cs, oidx[i]);
  }
  if (threadIdx.x == 0) {
    const int64_t gi = b * (int64_t)gridDim.x + tid;
    if (A.scale_bytes == 2) reinterpret_cast<uint16_t*>(A.s_out)[gi] = (uint16_t)g.sbits;
    else reinterpret_cast<uint8_t*>(A.s_out)[gi] = (uint8_t)g.sbits;
    if (A.zp_out) A.zp_out[gi] = (int8_t)g.zp;
  }
}

// ------------------------------------------------------------------ generic path
struct GenArgs {
  const uint16_t* w;
  int64_t batch, rows, cols, ld_row, ld_batch;
  int strategy;
  int64_t g;       // group size (GROUP / TENSOR_GROUP)
  int64_t bh, bw;  // BLOCK
  int64_t ng_item; // groups per batch item
  const float* col_scales;
  int64_t cs_ld_batch;  // col_scales stride between batch items (0: shared)
};

__device__ __forceinline__ int64_t group_of(const GenArgs& A, int64_t r, int64_t c) {
  switch (A.strategy) {
    case QZ_TENSOR: return 0;
    case QZ_CHANNEL: return r;
    case QZ_BLOCK: return (r / A.bh) * (A.cols / A.bw) + c / A.bw;
    default: return r * (A.cols / A.g) + c / A.g;
  }
}

__device__ __forceinline__ float load_w(const GenArgs& A, int64_t b, int64_t r, int64_t c) {
  float x = bf2f(A.w[b * A.ld_batch + r * A.ld_row + c]);
  if (A.col_scales) x = bfr(x * A.col_scales[b * A.cs_ld_batch + c]);
  return x;
}

__global__ void k_fill_u32(uint32_t* p, int64_t n, uint32_t v) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// one workgroup per (group, split): reduce the group's region, merge with key atomics
__global__ __launch_bounds__(BLOCK) void k_minmax_generic(GenArgs A, uint32_t* kmin, uint32_t* kmax) {
  const int64_t gi = blockIdx.x;  // global group id
  const int64_t b = gi / A.ng_item, gl = gi % A.ng_item;
  int64_t r0, r1, c0, c1;
  switch (A.strategy) {
    case QZ_TENSOR: {
      const int64_t ny = gridDim.y;
      r0 = A.rows * blockIdx.y / ny;
      r1 = A.rows * (blockIdx.y + 1) / ny;
      c0 = 0; c1 = A.cols;
      break;
    }
    case QZ_CHANNEL: r0 = gl; r1 = gl + 1; c0 = 0; c1 = A.cols; break;
    case QZ_BLOCK: {
      const int64_t nbc = A.cols / A.bw;
      r0 = (gl / nbc) * A.bh; r1 = r0 + A.bh;
      c0 = (gl % nbc) * A.bw; c1 = c0 + A.bw;
      break;
    }
    default: {
      const int64_t gpr = A.cols / A.g;
      r0 = gl / gpr; r1 = r0 + 1;
      c0 = (gl % gpr) * A.g; c1 = c0 + A.g;
    }
  }
  float mn = INFINITY, mx = -INFINITY;
  const int64_t width = c1 - c0;
  const int64_t n = (r1 - r0) * width;
  for (int64_t i = threadIdx.x; i < n; i += BLOCK) {
    const int64_t r = r0 + i / width, c = c0 + i % width;
    const float x = load_w(A, b, r, c);
    mn = fminf(mn, x);
    mx = fmaxf(mx, x);
  }
  mn = grp_min<WAVE>(mn);
  mx = grp_max<WAVE>(mx);
  __shared__ float smn[BLOCK / WAVE], smx[BLOCK / WAVE];
  if ((threadIdx.x & 63) == 0) { smn[threadIdx.x >> 6] = mn; smx[threadIdx.x >> 6] = mx; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < BLOCK / WAVE; ++k) { mn = fminf(mn, smn[k]); mx = fmaxf(mx, smx[k]); }
    if (n > 0) {
      atomicMin(&kmin[gi], f2key(mn));
      atomicMax(&kmax[gi], f2key(mx));
    }
  }
}

// NVFP4 global scale per batch item: (448*6)/absmax in bf16 as reciprocal-then-multiply
// (python-scalar / tensor == tensor.reciprocal() * scalar), then widened to f32.
// Per-slice |w| maximum (NVFP4's per-tensor observer) for dense, 16-B aligned slices: 16-B
// loads, 4 in flight per lane, v_pk_max_u16 on |bf16| bit patterns, wave DPP max, one atomic per
// workgroup.  tmin/tmax receive the keys of -absmax / +absmax (all k_gscale_keys needs).
__global__ __launch_bounds__(256) void k_absmax_slices(const uint16_t* w, int64_t units_per_batch, int64_t ld_batch,
                                                       uint32_t* tmin, uint32_t* tmax) {
  const int64_t b = blockIdx.y;
  const uint4* src = reinterpret_cast<const uint4*>(w + b * ld_batch);
  const int64_t stride = (int64_t)gridDim.x * 256;
  uint32_t m = 0;
  int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; u + 3 * stride < units_per_batch; u += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // read-once stream: non-temporal
      const u32x4 t = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + u + j * stride));
      v[j] = make_uint4(t.x, t.y, t.z, t.w);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      m = pk_max_u16(m, pk_max_u16(pk_max_u16(v[j].x & 0x7fff7fffu, v[j].y & 0x7fff7fffu),
                                   pk_max_u16(v[j].z & 0x7fff7fffu, v[j].w & 0x7fff7fffu)));
  }
  for (; u < units_per_batch; u += stride) {
    const uint4 v = src[u];
    m = pk_max_u16(m, pk_max_u16(pk_max_u16(v.x & 0x7fff7fffu, v.y & 0x7fff7fffu),
                                 pk_max_u16(v.z & 0x7fff7fffu, v.w & 0x7fff7fffu)));
  }
  m = grp_max_u<WAVE>(max(m & 0xffffu, m >> 16));
  __shared__ uint32_t red[256 / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) red[threadIdx.x / WAVE] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = max(max(red[0], red[1]), max(red[2], red[3]));
    const float am = __uint_as_float(m << 16);
    atomicMax(tmax + b, f2key(am));
    atomicMin(tmin + b, f2key(-am));
  }
}

__global__ void k_gscale_keys(const uint32_t* tmin, const uint32_t* tmax, int64_t batch, float* gs) {
  int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= batch) return;
  float lo = fminf(key2f(tmin[b]), 0.f), hi = fmaxf(key2f(tmax[b]), 0.f);
  float am = fmaxf(fabsf(lo), fabsf(hi));
  gs[b] = bfr(bfr(1.0f / am) * 2688.0f);
}

// ------------------------------------------------------------ NVFP4 fused path (round 4)
// NVFP4 (TENSOR_GROUP) needs each slice's |w| maximum (its global scale) before any group of
// that slice can be encoded.  Two launches, no fills and no separate global-scale launch:
// k_nv_absmax reduces 32 KiB tiles of every slice into the slice's key (agent-scope atomic max of
// the |bf16| bits, executed at the memory side), k_nv_encode re-reads each tile, forms the global
// scale from the key (the launch boundary orders the first launch's atomics before it), encodes
// and stores codes, e4m3 scales and the global scale; the last tile of a slice to finish resets
// the slice's key and tile count, so the sync region is zero after every call (caller contract:
// zero before the first call).  HBM traffic = two reads + one write; a fused Qwen3-30B-A3B expert
// parameter (403 MB) does not fit the 256 MiB MALL, so no chunking makes the second read cheaper
// (chunked, register-held and single-launch variants were measured and removed).
constexpr int NV_BLOCK = 256;
constexpr int NV_U = 8;                                   // units (8 bf16) per lane per tile
constexpr int64_t NV_TILE = (int64_t)NV_BLOCK * NV_U;     // 2048 units = 32 KiB of bf16 per workgroup
constexpr int NV_SYNC_STRIDE = 16;                        // uint32 words per slice: {key, tile count}, one 64-B line

struct NvArgs {
  const uint64_t* tab;  // table mode: DEVICE [4][n_slices] {weight, codes, scales, global scale}; null = batch mode
  const uint16_t* w;    // batch mode: slice b at w + b * ld_batch (elements), dense rows
  int64_t ld_batch;
  void* q_out;          // batch mode outputs, dense batch-major
  void* s_out;
  float* gs_out;
  int64_t n_slices;
  int64_t units_per_slice;  // rows * cols / 8
  int64_t tiles_per_slice;
  uint32_t* sync;           // [n_slices][NV_SYNC_STRIDE]
  QP p;
};

// A sync word read AT THE MEMORY SIDE, by a compare-exchange that always fails (a key never holds
// all ones): a relaxed agent-scope atomic load, or an idempotent RMW (which LLVM turns into one),
// compiles to a global_load ... sc1 that can be served from this XCD's L2 copy of the line while
// other XCDs' atomics update it (per-XCD L2s are not coherent).
__device__ __forceinline__ uint32_t sync_read(uint32_t* p) {
  uint32_t e = 0xffffffffu;
  __hip_atomic_compare_exchange_strong(p, &e, 0xfffffffeu, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
  return e;
}

__device__ __forceinline__ uint32_t absmax_bits(const uint4 v) {
  return pk_max_u16(pk_max_u16(v.x & 0x7fff7fffu, v.y & 0x7fff7fffu), pk_max_u16(v.z & 0x7fff7fffu, v.w & 0x7fff7fffu));
}

template <bool TAB>
__device__ __forceinline__ const uint4* nv_slice(const NvArgs& A, int64_t b) {
  return TAB ? reinterpret_cast<const uint4*>(A.tab[b]) : reinterpret_cast<const uint4*>(A.w + b * A.ld_batch);
}

// one tile's units, non-temporal (each launch reads a line once); lanes past the slice's end
// re-read its last unit
__device__ __forceinline__ void nv_load(uint4 (&v)[NV_U], const uint4* src, int64_t base, int64_t ups, int tid) {
#pragma unroll
  for (int u = 0; u < NV_U; ++u) {
    const int64_t un = min<int64_t>(base + u * NV_BLOCK + tid, ups - 1);
    v[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + un)));
  }
}

template <bool TAB>
__global__ __launch_bounds__(NV_BLOCK) void k_nv_absmax(NvArgs A) {
  __shared__ uint32_t red[NV_BLOCK / WAVE];
  const int tid = threadIdx.x, lane = tid & (WAVE - 1), wv = tid >> 6;
  const int64_t b = blockIdx.x / A.tiles_per_slice, base = (blockIdx.x % A.tiles_per_slice) * NV_TILE;
  uint4 v[NV_U];
  nv_load(v, nv_slice<TAB>(A, b), base, A.units_per_slice, tid);
  uint32_t m = 0;
#pragma unroll
  for (int u = 0; u < NV_U; ++u) m = pk_max_u16(m, absmax_bits(v[u]));
  m = grp_max_u<WAVE>(max(m & 0xffffu, m >> 16));
  if (lane == 0) red[wv] = m;
  __syncthreads();
  if (tid == 0)
    __hip_atomic_fetch_max(A.sync + NV_SYNC_STRIDE * b, max(max(red[0], red[1]), max(red[2], red[3])),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One unit (8 bf16; a group of 16 = two lanes) of a slice with a finite global scale: the
// arithmetic of group_params(K_NV) + encode_store, with (a) the e4m3 scale code from
// v_cvt_pk_fp8_f32 (RNE; the FP8 path's conversion, exhaustively checked on bf16 inputs: s32 =
// gs * s is an exact product of two bf16 in [0, 448]) and (b) the code's dense scale sf / gs and
// its reciprocal from the workgroup's 128-entry tables (ts, trs: the same IEEE division and rcp,
// done once per code instead of once per group; trs = 0 where the rcp is not accurate, which sends
// every element of the group to the IEEE division, as g.fast == false does).  A per-unit instead of
// per-pair boundary branch in encode_store measured slower (158 vs 150 us per [128, 768, 2048],
// profiles/r04n_nvprobe_*.log).
__device__ __forceinline__ void nv_unit(const FastArgs& F, const QP& p, const uint4 v, int64_t unit, bool valid,
                                        float gs, int lane, const float* ts, const float* trs) {
  const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
  f32x2 x[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    x[k].x = __uint_as_float(wd[k] << 16);
    x[k].y = __uint_as_float(wd[k] & 0xffff0000u);
  }
  const uint32_t m = pk_max_u16(pk_max_u16(wd[0] & 0x7fff7fffu, wd[1] & 0x7fff7fffu),
                                pk_max_u16(wd[2] & 0x7fff7fffu, wd[3] & 0x7fff7fffu));
  const float am = __uint_as_float(grp_max_u<2>(max(m & 0xffffu, m >> 16) << 16));
  const float s = (am == 0.f) ? 0.f : bf16_quot(am, p.half_range, p.inv_half);
  uint32_t s8 = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(fminf(gs * s, 448.f), 0.f, 0, false) & 0xffu;
  if (s8 == 0) s8 = 0x20u;  // eps of float8_e4m3fn (D1)
  GP g;
  g.sbits = s8;
  g.s = ts[s8];
  g.rs = trs[s8];
  g.zp = 0.f;
  g.fast = true;
  if (!valid) return;
  encode_store<K_NV, false, true, true>(F, p, g, x, nullptr, unit);
  if ((lane & 1) == 0) reinterpret_cast<uint8_t*>(F.s_out)[unit >> 1] = (uint8_t)s8;
}

template <bool TAB>
__global__ __launch_bounds__(NV_BLOCK) void k_nv_encode(NvArgs A) {
  __shared__ uint32_t keysh;
  const int tid = threadIdx.x, lane = tid & (WAVE - 1);
  const int64_t b = blockIdx.x / A.tiles_per_slice, base = (blockIdx.x % A.tiles_per_slice) * NV_TILE;
  const int64_t ups = A.units_per_slice;
  uint32_t* sy = A.sync + NV_SYNC_STRIDE * b;
  uint4 v[NV_U];
  nv_load(v, nv_slice<TAB>(A, b), base, ups, tid);
  if (tid == 0) keysh = sync_read(sy);  // final: k_nv_absmax finished before this launch began
  __syncthreads();
  QP p = A.p;
  p.kind = K_NV;
  p.sym = 1;
  // global scale, k_gscale_keys' arithmetic: bf16(bf16(1 / absmax) * (448 * 6))
  const float gs = bfr(bfr(1.0f / __uint_as_float(keysh << 16)) * 2688.0f);
  FastArgs F;
  float* gs_out;
  if constexpr (TAB) {
    F.q_out = reinterpret_cast<void*>(A.tab[A.n_slices + b]);
    F.s_out = reinterpret_cast<void*>(A.tab[2 * A.n_slices + b]);
    gs_out = reinterpret_cast<float*>(A.tab[3 * A.n_slices + b]);
  } else {
    F.q_out = reinterpret_cast<uint32_t*>(A.q_out) + b * ups;
    F.s_out = reinterpret_cast<uint8_t*>(A.s_out) + b * (ups >> 1);
    gs_out = A.gs_out + b;
  }
  F.zp_out = nullptr;
  F.scale_bytes = 1;
  F.out_fmt = QZ_OUT_FP4_PACKED;
  F.col_scales = nullptr;
  if (base == 0 && tid == 0) *gs_out = gs;
  if (__builtin_isfinite(gs)) {  // workgroup-uniform
    __shared__ float ts[128], trs[128];
    if (tid < 128) {
      const float sc = e4m3_to_f32((uint32_t)tid) / gs;  // _quantize: scale / global_scale (f32)
      ts[tid] = sc;
      trs[tid] = (sc >= 0x1.0p-100f && sc <= 0x1.0p+100f) ? __builtin_amdgcn_rcpf(sc) : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < NV_U; ++u) {
      const int64_t local = base + u * NV_BLOCK + tid;
      nv_unit(F, p, v[u], local, local < ups, gs, lane, ts, trs);
    }
  } else {  // an all-zero (or non-finite) slice: the general arithmetic
#pragma unroll
    for (int u = 0; u < NV_U; ++u) {
      const int64_t local = base + u * NV_BLOCK + tid;
      process_unit<1, K_NV, false, true, true>(F, p, v[u], local, local < ups, gs, lane, 0, nullptr);
    }
  }
  if (tid == 0) {  // the slice's last tile resets its sync words for the next call
    const uint32_t old = __hip_atomic_fetch_add(sy + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (uint32_t)A.tiles_per_slice - 1u) {
      __hip_atomic_store(sy, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(sy + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ void store_qparams(const GP& g, int64_t gi, int scale_bytes, void* s_out, int8_t* zp_out) {
  if (scale_bytes == 2) reinterpret_cast<uint16_t*>(s_out)[gi] = (uint16_t)g.sbits;
  else reinterpret_cast<uint8_t*>(s_out)[gi] = (uint8_t)g.sbits;
  if (zp_out) zp_out[gi] = (int8_t)g.zp;
}

__global__ void k_qparams_keys(QP p, const uint32_t* kmin, const uint32_t* kmax, int64_t ng,
                               int64_t ng_item, const float* gscale, int scale_bytes, void* s_out,
                               int8_t* zp_out) {
  int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= ng) return;
  float gs = (p.kind == K_NV) ? gscale[gi / ng_item] : 0.f;
  GP g = group_params(p, key2f(kmin[gi]), key2f(kmax[gi]), gs);
  store_qparams(g, gi, scale_bytes, s_out, zp_out);
}

__global__ void k_qparams_bf16(QP p, const uint16_t* mn, const uint16_t* mx, int64_t n,
                               const float* gscale, int scale_bytes, void* s_out, int8_t* zp_out) {
  int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (gi >= n) return;
  float gs = (p.kind == K_NV) ? gscale[0] : 0.f;
  GP g = group_params(p, bf2f(mn[gi]), bf2f(mx[gi]), gs);
  store_qparams(g, gi, scale_bytes, s_out, zp_out);
}

__global__ void k_keys_to_bf16(const uint32_t* kmin, const uint32_t* kmax, int64_t n, uint16_t* mn, uint16_t* mx) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  mn[i] = f2bf(key2f(kmin[i]));
  mx[i] = f2bf(key2f(kmax[i]));
}

// one thread per output item (packed word / fp4 byte / element)
__global__ void k_quant_generic(GenArgs A, QP p, int out_fmt, int scale_fmt, const void* scale,
                                const int8_t* zp, const float* gscale, void* q_out, int64_t items_per_row,
                                int64_t elems_per_item) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = A.batch * A.rows * items_per_row;
  if (idx >= total) return;
  const int64_t brow = idx / items_per_row, it = idx % items_per_row;
  const int64_t b = brow / A.rows, r = brow % A.rows;
  const float gs = (p.kind == K_NV) ? gscale[b] : 0.f;
  uint32_t word = 0;
  for (int64_t i = 0; i < elems_per_item; ++i) {
    const int64_t c = it * elems_per_item + i;
    if (c >= A.cols) break;
    const int64_t gi = b * A.ng_item + group_of(A, r, c);
    const GP g = gp_from_stored(p, scale_fmt, scale, gi, zp, gs);
    const float x = load_w(A, b, r, c);
    const uint32_t code = encode(p, g, x);
    const int64_t e = brow * A.cols + c;  // dense element index
    if (out_fmt == QZ_OUT_FAKEQUANT) {
      float d = (p.kind == K_INT) ? fakequant_int(p, g, x) : decode(p, g, code);
      if (A.col_scales) d = bfr(d / A.col_scales[b * A.cs_ld_batch + c]);
      reinterpret_cast<uint16_t*>(q_out)[e] = f2bf(d);
    } else if (out_fmt == QZ_OUT_INT8) {
      reinterpret_cast<int8_t*>(q_out)[e] = (int8_t)((int)code + (int)p.qmin);
    } else if (out_fmt == QZ_OUT_FP8) {
      reinterpret_cast<uint8_t*>(q_out)[e] = (uint8_t)code;
    } else if (out_fmt == QZ_OUT_FP4_PACKED) {
      word |= code << (4 * i);
    } else {  // PACKED_INT32
      word |= code << (p.bits * i);
    }
  }
  if (out_fmt == QZ_OUT_PACKED_INT32) reinterpret_cast<uint32_t*>(q_out)[idx] = word;
  else if (out_fmt == QZ_OUT_FP4_PACKED) reinterpret_cast<uint8_t*>(q_out)[idx] = (uint8_t)word;
}

__global__ void k_dequant_generic(const void* q, int64_t batch, int64_t rows, int64_t cols, QP p, int in_fmt,
                                  GenArgs A, int scale_fmt, const void* scale, const int8_t* zp,
                                  const float* gscale, uint16_t* out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= batch * rows * cols) return;
  const int64_t brow = e / cols, c = e % cols;
  const int64_t b = brow / rows, r = brow % rows;
  uint32_t code;
  if (in_fmt == QZ_OUT_PACKED_INT32) {
    const int pf = 32 / p.bits;
    const int64_t wpr = (cols + pf - 1) / pf;
    const uint32_t word = reinterpret_cast<const uint32_t*>(q)[brow * wpr + c / pf];
    code = (word >> (p.bits * (c % pf))) & ((1u << p.bits) - 1u);
  } else if (in_fmt == QZ_OUT_INT8) {
    code = (uint32_t)((int)reinterpret_cast<const int8_t*>(q)[e] - (int)p.qmin);
  } else if (in_fmt == QZ_OUT_FP8) {
    code = reinterpret_cast<const uint8_t*>(q)[e];
  } else {
    const uint8_t byte = reinterpret_cast<const uint8_t*>(q)[e >> 1];
    code = (e & 1) ? (byte >> 4) : (byte & 15u);
  }
  const float gs = (p.kind == K_NV) ? gscale[b] : 0.f;
  const int64_t gi = b * A.ng_item + group_of(A, r, c);
  const GP g = gp_from_stored(p, scale_fmt, scale, gi, zp, gs);
  out[e] = f2bf(decode(p, g, code));
}

__global__ void k_pack_int32(const int8_t* v, int64_t rows, int64_t cols, int bits, int packed_dim, int32_t* out) {
  const int pf = 32 / bits;
  const uint32_t mask = (1u << bits) - 1u;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (packed_dim == 1) {
    const int64_t wpr = (cols + pf - 1) / pf;
    if (idx >= rows * wpr) return;
    const int64_t r = idx / wpr, j = idx % wpr;
    uint32_t word = 0;
    for (int i = 0; i < pf; ++i) {
      const int64_t c = j * pf + i;
      if (c < cols) word |= ((uint32_t)(v[r * cols + c] + (1 << (bits - 1))) & mask) << (bits * i);
    }
    out[idx] = (int32_t)word;
  } else {
    const int64_t h = (rows + pf - 1) / pf;
    if (idx >= h * cols) return;
    const int64_t j = idx / cols, c = idx % cols;
    uint32_t word = 0;
    for (int i = 0; i < pf; ++i) {
      const int64_t r = j * pf + i;
      if (r < rows) word |= ((uint32_t)(v[r * cols + c] + (1 << (bits - 1))) & mask) << (bits * i);
    }
    out[idx] = (int32_t)word;
  }
}

// ---------------------------------------------------------------------- host side
using FastFn = void (*)(FastArgs);

// fq: AWQ fake-quant; nt: non-temporal weight stream (launches much larger than the 256 MiB
// Infinity Cache: the read-once weight should not evict the outputs; +6 % at 360 MB, -2 % at 90 MB)
// grp: grouped launch over a device pointer table (quantize only; NVFP4 needs its per-tensor pass)
template <int LOGL, int KIND, bool SYM>
FastFn pick_fq(bool fq, bool nt, bool grp) {
  if constexpr (KIND != K_NV) {
    if (grp) return nt ? (FastFn)k_group_fast<LOGL, KIND, false, SYM, true, true>
                       : (FastFn)k_group_fast<LOGL, KIND, false, SYM, false, true>;
  }
  if (fq) return nt ? (FastFn)k_group_fast<LOGL, KIND, true, SYM, true> : (FastFn)k_group_fast<LOGL, KIND, true, SYM>;
  return nt ? (FastFn)k_group_fast<LOGL, KIND, false, SYM, true> : (FastFn)k_group_fast<LOGL, KIND, false, SYM>;
}
template <int LOGL>
FastFn pick_kind(int kind, bool sym, bool fq, bool nt, bool grp) {
  switch (kind) {
    case K_INT: return sym ? pick_fq<LOGL, K_INT, true>(fq, nt, grp) : pick_fq<LOGL, K_INT, false>(fq, nt, grp);
    case K_FP8: return pick_fq<LOGL, K_FP8, true>(fq, nt, grp);
    case K_MX: return pick_fq<LOGL, K_MX, true>(fq, nt, grp);
    case K_NV: return pick_fq<LOGL, K_NV, true>(fq, nt, grp);
    default: return pick_fq<LOGL, K_FP4, true>(fq, nt, grp);
  }
}
FastFn pick_fast(int logl, int kind, bool sym, bool fq, bool nt, bool grp = false) {
  switch (logl) {
    case 0: return pick_kind<0>(kind, sym, fq, nt, grp);
    case 1: return pick_kind<1>(kind, sym, fq, nt, grp);
    case 2: return pick_kind<2>(kind, sym, fq, nt, grp);
    case 3: return pick_kind<3>(kind, sym, fq, nt, grp);
    case 4: return pick_kind<4>(kind, sym, fq, nt, grp);
    case 5: return pick_kind<5>(kind, sym, fq, nt, grp);
    default: return pick_kind<6>(kind, sym, fq, nt, grp);
  }
}

using FqcFn = void (*)(FastArgs, int64_t);
template <int LOGL, bool NT>
FqcFn pick_fqc_kind(int kind, bool sym) {
  switch (kind) {
    case K_INT: return sym ? (FqcFn)k_fq_cols<LOGL, K_INT, true, NT> : (FqcFn)k_fq_cols<LOGL, K_INT, false, NT>;
    case K_FP8: return k_fq_cols<LOGL, K_FP8, true, NT>;
    case K_MX: return k_fq_cols<LOGL, K_MX, true, NT>;
    case K_FP4: return k_fq_cols<LOGL, K_FP4, true, NT>;
    default: return nullptr;  // NVFP4: unit-wise kernel (needs the per-tensor pre-pass)
  }
}
template <bool NT>
FqcFn pick_fqc_nt(int logl, int kind, bool sym) {
  switch (logl) {
    case 0: return pick_fqc_kind<0, NT>(kind, sym);
    case 1: return pick_fqc_kind<1, NT>(kind, sym);
    case 2: return pick_fqc_kind<2, NT>(kind, sym);
    case 3: return pick_fqc_kind<3, NT>(kind, sym);
    case 4: return pick_fqc_kind<4, NT>(kind, sym);
    case 5: return pick_fqc_kind<5, NT>(kind, sym);
    default: return pick_fqc_kind<6, NT>(kind, sym);
  }
}
FqcFn pick_fqc(int logl, int kind, bool sym, bool nt) {
  return nt ? pick_fqc_nt<true>(logl, kind, sym) : pick_fqc_nt<false>(logl, kind, sym);
}

using TileFn = void (*)(FastArgs, TileArgs);
template <int KIND, bool SYM, bool NT>
TileFn pick_tile_u(int maxu) {
  switch (maxu) {
    case 1: return k_tile_fast<KIND, SYM, 1, NT>;
    case 2: return k_tile_fast<KIND, SYM, 2, NT>;
    case 4: return k_tile_fast<KIND, SYM, 4, NT>;
    case 8: return k_tile_fast<KIND, SYM, 8, NT>;
    default: return k_tile_fast<KIND, SYM, 16, NT>;
  }
}
template <bool NT>
TileFn pick_tile_nt(int kind, bool sym, int maxu) {
  switch (kind) {
    case K_INT: return sym ? pick_tile_u<K_INT, true, NT>(maxu) : pick_tile_u<K_INT, false, NT>(maxu);
    case K_FP8: return pick_tile_u<K_FP8, true, NT>(maxu);
    default: return pick_tile_u<K_FP4, true, NT>(maxu);
  }
}
TileFn pick_tile(int kind, bool sym, int maxu, bool nt) {
  return nt ? pick_tile_nt<true>(kind, sym, maxu) : pick_tile_nt<false>(kind, sym, maxu);
}

struct Plan {
  QP p;
  int kind;
  int scale_fmt;
  int scale_bytes;
  int64_t ng_item;  // groups per batch item
};

int make_plan(const qz_args* a, int64_t rows, int64_t cols, Plan* pl) {
  if (!a) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0) return QZ_ERR_SHAPE;
  QP& p = pl->p;
  p.sym = a->symmetric ? 1 : 0;
  p.bits = a->num_bits;
  if (a->type == QZ_INT) {
    if (a->num_bits < 2 || a->num_bits > 8) return QZ_ERR_BITS;
    if (a->scale_fmt != QZ_SCALE_NATIVE) return QZ_ERR_FORMAT;
    p.qmin = -(float)(1 << (a->num_bits - 1));
    p.qmax = (float)((1 << (a->num_bits - 1)) - 1);
    pl->kind = K_INT;
  } else if (a->type == QZ_FLOAT) {
    if (!a->symmetric) return QZ_ERR_ASYM_FLOAT;
    if (a->num_bits == 8) {
      if (a->scale_fmt != QZ_SCALE_NATIVE) return QZ_ERR_FORMAT;
      p.qmin = -448.f; p.qmax = 448.f; pl->kind = K_FP8;
    } else if (a->num_bits == 4) {
      p.qmin = -6.f; p.qmax = 6.f;
      if (a->scale_fmt == QZ_SCALE_E8M0) pl->kind = K_MX;
      else if (a->strategy == QZ_TENSOR_GROUP) {
        if (a->scale_fmt != QZ_SCALE_E4M3) return QZ_ERR_FORMAT;
        pl->kind = K_NV;
      } else if (a->scale_fmt == QZ_SCALE_NATIVE) pl->kind = K_FP4;
      else return QZ_ERR_FORMAT;
    } else return QZ_ERR_BITS;
  } else return QZ_ERR_FORMAT;
  p.kind = pl->kind;
  p.half_range = (p.qmax - p.qmin) / 2.0f;
  p.range = p.qmax - p.qmin;
  p.inv_half = 1.0f / p.half_range;
  p.inv_range = 1.0f / p.range;
  p.magic = 8388608.0f - p.qmin;
  pl->scale_fmt = a->scale_fmt;
  pl->scale_bytes = (a->scale_fmt == QZ_SCALE_NATIVE) ? 2 : 1;
  switch (a->strategy) {
    case QZ_TENSOR: pl->ng_item = 1; break;
    case QZ_CHANNEL: pl->ng_item = rows; break;
    case QZ_GROUP:
    case QZ_TENSOR_GROUP:
      if (a->group_size <= 0 || cols % a->group_size) return QZ_ERR_GROUP;
      if (pl->kind == K_MX && a->strategy != QZ_GROUP) return QZ_ERR_FORMAT;
      pl->ng_item = rows * (cols / a->group_size);
      break;
    case QZ_BLOCK:
      if (a->block_h <= 0 || a->block_w <= 0 || rows % a->block_h || cols % a->block_w) return QZ_ERR_BLOCK;
      pl->ng_item = (rows / a->block_h) * (cols / a->block_w);
      break;
    default: return QZ_ERR_FORMAT;
  }
  if (pl->kind == K_NV && a->strategy != QZ_TENSOR_GROUP) return QZ_ERR_FORMAT;
  return QZ_OK;
}

int check_out_fmt(const Plan& pl, int out_fmt) {
  switch (out_fmt) {
    case QZ_OUT_PACKED_INT32: return pl.kind == K_INT ? QZ_OK : QZ_ERR_FORMAT;
    case QZ_OUT_INT8: return pl.kind == K_INT ? QZ_OK : QZ_ERR_FORMAT;
    case QZ_OUT_FP8: return pl.kind == K_FP8 ? QZ_OK : QZ_ERR_FORMAT;
    case QZ_OUT_FP4_PACKED: return (pl.kind == K_MX || pl.kind == K_NV || pl.kind == K_FP4) ? QZ_OK : QZ_ERR_FORMAT;
    case QZ_OUT_FAKEQUANT: return QZ_OK;
  }
  return QZ_ERR_FORMAT;
}

GenArgs gen_args(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row, int64_t ld_batch,
                 const qz_args* a, const Plan& pl, const float* col_scales, int64_t cs_ld_batch = 0) {
  GenArgs G;
  G.w = (const uint16_t*)w;
  G.batch = batch; G.rows = rows; G.cols = cols; G.ld_row = ld_row; G.ld_batch = ld_batch;
  G.strategy = a->strategy;
  G.g = a->group_size > 0 ? a->group_size : cols;
  G.bh = a->block_h; G.bw = a->block_w;
  G.ng_item = pl.ng_item;
  G.col_scales = col_scales;
  G.cs_ld_batch = cs_ld_batch;
  return G;
}

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline bool aligned(const void* p, size_t n) { return ((uintptr_t)p % n) == 0; }

int launch_err() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QZ_OK : (int)e;
}

// reduce per-group (or per-tensor) min/max keys into ws: kmin[ng], kmax[ng]
int run_minmax(const GenArgs& G, int64_t ng_total, uint32_t* kmin, uint32_t* kmax, hipStream_t st) {
  const int64_t nb = cdiv(ng_total, 256);
  hipLaunchKernelGGL(k_fill_u32, dim3((unsigned)nb), dim3(256), 0, st, kmin, ng_total, 0xffffffffu);
  hipLaunchKernelGGL(k_fill_u32, dim3((unsigned)nb), dim3(256), 0, st, kmax, ng_total, 0u);
  dim3 grid((unsigned)ng_total, 1);
  if (G.strategy == QZ_TENSOR) {
    const int64_t elems = G.rows * G.cols;
    grid.y = (unsigned)std::min<int64_t>(std::max<int64_t>(1, elems / (BLOCK * 64)), std::min<int64_t>(G.rows, 4096));
  }
  hipLaunchKernelGGL(k_minmax_generic, grid, dim3(BLOCK), 0, st, G, kmin, kmax);
  return launch_err();
}

// workspace layout (all regions 256-B aligned):
//   kmin[ng] u32 | kmax[ng] u32 | tmin[batch] u32 | tmax[batch] u32 |
//   scale[ng] (2 B) | zp[ng] (1 B) | gscale[batch] f32
struct WS {
  uint32_t *kmin, *kmax, *tmin, *tmax;
  void* scale;
  int8_t* zp;
  float* gscale;
  size_t bytes;
};
inline size_t al256(size_t n) { return (n + 255) & ~(size_t)255; }
WS ws_layout(void* base, int64_t batch, const Plan& pl) {
  const size_t ng = (size_t)(batch * pl.ng_item);
  WS w;
  char* p = (char*)base;
  size_t off = 0;
  w.kmin = (uint32_t*)(p + off); off += al256(4 * ng);
  w.kmax = (uint32_t*)(p + off); off += al256(4 * ng);
  w.tmin = (uint32_t*)(p + off); off += al256(4 * (size_t)batch);
  w.tmax = (uint32_t*)(p + off); off += al256(4 * (size_t)batch);
  w.scale = (void*)(p + off); off += al256(2 * ng);
  w.zp = (int8_t*)(p + off); off += al256(ng);
  w.gscale = (float*)(p + off); off += al256(4 * (size_t)batch);
  w.bytes = off;
  return w;
}
size_t ws_size(int64_t batch, const Plan& pl) { return ws_layout(nullptr, batch, pl).bytes; }

int nv_args_ok(const qz_args* a, int64_t rows, int64_t cols, Plan* pl) {
  if (!a) return QZ_ERR_NULL;
  int rc = make_plan(a, rows, cols, pl);
  if (rc) return rc;
  if (pl->kind != K_NV || a->group_size != 16) return QZ_ERR_FORMAT;
  return QZ_OK;
}

int nv_launch(NvArgs& A, bool tab, void* sync, size_t sync_bytes, hipStream_t st) {
  if (!sync) return QZ_ERR_NULL;
  if (!aligned(sync, 16)) return QZ_ERR_ALIGN;
  if (sync_bytes < 4 * NV_SYNC_STRIDE * (size_t)A.n_slices) return QZ_ERR_WORKSPACE;
  A.sync = (uint32_t*)sync;
  A.tiles_per_slice = cdiv(A.units_per_slice, NV_TILE);
  const int64_t grid = A.n_slices * A.tiles_per_slice;
  if (grid > 0x7fffffffLL) return QZ_ERR_SHAPE;
  if (tab) hipLaunchKernelGGL(k_nv_absmax<true>, dim3((unsigned)grid), dim3(NV_BLOCK), 0, st, A);
  else hipLaunchKernelGGL(k_nv_absmax<false>, dim3((unsigned)grid), dim3(NV_BLOCK), 0, st, A);
  int rc = launch_err();
  if (rc) return rc;
  if (tab) hipLaunchKernelGGL(k_nv_encode<true>, dim3((unsigned)grid), dim3(NV_BLOCK), 0, st, A);
  else hipLaunchKernelGGL(k_nv_encode<false>, dim3((unsigned)grid), dim3(NV_BLOCK), 0, st, A);
  rc = launch_err();
  // the |w| max launch has run but the encode (which resets the sync lines) has not: clear them,
  // so the region is zero for the next call on this stream as the contract says
  if (rc) (void)hipMemsetAsync(A.sync, 0, 4 * NV_SYNC_STRIDE * (size_t)A.n_slices, st);
  return rc;
}

}  // namespace

extern "C" {

const char* qz_strerror(int code) {
  switch (code) {
    case QZ_OK: return "ok";
    case QZ_ERR_NULL: return "required pointer is NULL";
    case QZ_ERR_SHAPE: return "invalid shape";
    case QZ_ERR_GROUP: return "tensor column shape must be divisible by the given group_size";
    case QZ_ERR_BLOCK: return "Block quantization requires exact division";
    case QZ_ERR_BITS: return "num_bits not supported for this type / format";
    case QZ_ERR_ASYM_FLOAT: return "Asymmetric Quantization is not supported for float types";
    case QZ_ERR_FORMAT: return "output/scale format incompatible with the quantization args";
    case QZ_ERR_WORKSPACE: return "workspace too small";
    case QZ_ERR_ALIGN: return "alignment requirement violated";
    case QZ_ERR_UNAVAILABLE: return "runtime dependency unavailable (hipBLASLt not loaded or refused the call)";
  }
  return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown error";
}

int qz_version(void) { return 200; }

const char* qz_build_config(void) {
  // the constants above (k_group_fast's NT instantiation = weight bytes > nt_bytes_q)
  return "nt_bytes_q=0;nt_bytes_fq=268435456;unroll=2;unroll_nt=2;fast_block=128;reg_loads=0;reg_loads_grp=1;"
         "arch=gfx950";
}

size_t qz_quantize_workspace_size(int64_t batch, int64_t rows, int64_t cols, const qz_args* a) {
  Plan pl;
  if (make_plan(a, rows, cols, &pl) != QZ_OK) return 0;
  return ws_size(batch, pl);
}

static int quantize_impl(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row,
                         int64_t ld_batch, const qz_args* a, int32_t out_fmt, void* q_out, void* scale_out,
                         int8_t* zp_out, float* gscale_out, const float* col_scales, int64_t cs_ld_batch,
                         void* ws, size_t ws_bytes, hipStream_t st) {
  if (!w || !q_out || !a) return QZ_ERR_NULL;
  if (batch <= 0) return QZ_ERR_SHAPE;
  Plan pl;
  int rc = make_plan(a, rows, cols, &pl);
  if (rc) return rc;
  if ((rc = check_out_fmt(pl, out_fmt))) return rc;
  if (out_fmt != QZ_OUT_FAKEQUANT && !scale_out) return QZ_ERR_NULL;
  if (out_fmt != QZ_OUT_FAKEQUANT && pl.kind == K_NV && !gscale_out) return QZ_ERR_NULL;
  if (ld_row < cols || (batch > 1 && ld_batch < rows * ld_row)) return QZ_ERR_SHAPE;
  const bool fq = out_fmt == QZ_OUT_FAKEQUANT;
  const int64_t ng = batch * pl.ng_item;
  if (!ws || ws_bytes < ws_size(batch, pl)) return QZ_ERR_WORKSPACE;
  const WS W = ws_layout(ws, batch, pl);
  const bool contig = ld_row == cols && (batch == 1 || ld_batch == rows * cols);
  const bool rows_dense = ld_row == cols && (batch == 1 || ld_batch % 8 == 0);  // fast path: per-slice dense
  if (fq && q_out == w && !contig) return QZ_ERR_FORMAT;  // in place only when dense
  // fake-quant keeps its qparams in the workspace
  void* s_dst = scale_out ? scale_out : W.scale;
  int8_t* z_dst = scale_out ? zp_out : W.zp;
  if (!pl.p.sym && !z_dst) z_dst = W.zp;
  float* gs_dst = gscale_out ? gscale_out : W.gscale;

  if (col_scales && cs_ld_batch != 0 && cs_ld_batch < cols) return QZ_ERR_SHAPE;
  GenArgs G = gen_args(w, batch, rows, cols, ld_row, ld_batch, a, pl, col_scales, cs_ld_batch);

  // NVFP4: per-tensor global scale first
  if (pl.kind == K_NV) {
    GenArgs T = G;
    T.strategy = QZ_TENSOR;
    T.ng_item = 1;
    if (!col_scales && rows_dense && aligned(w, 16) && cols % 8 == 0 && (batch == 1 || ld_batch % 8 == 0) &&
        batch <= 65535) {  // (AWQ's fake-quant observes W * s: generic path)
      const int64_t ups = rows * cols / 8;
      const int64_t chunks = std::max<int64_t>(1, std::min<int64_t>(cdiv(ups, 256 * 4), cdiv(2048, batch)));
      hipLaunchKernelGGL(k_fill_u32, dim3((unsigned)cdiv(batch, 256)), dim3(256), 0, st, W.tmin, batch, 0xffffffffu);
      hipLaunchKernelGGL(k_fill_u32, dim3((unsigned)cdiv(batch, 256)), dim3(256), 0, st, W.tmax, batch, 0u);
      hipLaunchKernelGGL(k_absmax_slices, dim3((unsigned)chunks, (unsigned)batch), dim3(256), 0, st,
                         (const uint16_t*)w, ups, batch > 1 ? ld_batch : rows * cols, W.tmin, W.tmax);
    } else if ((rc = run_minmax(T, batch, W.tmin, W.tmax, st))) {
      return rc;
    }
    hipLaunchKernelGGL(k_gscale_keys, dim3((unsigned)cdiv(batch, 64)), dim3(64), 0, st, W.tmin, W.tmax, batch, gs_dst);
    if ((rc = launch_err())) return rc;
  }

  const int64_t g = a->group_size;
  const bool grp = a->strategy == QZ_GROUP || a->strategy == QZ_TENSOR_GROUP;
  const bool pow2 = g >= 8 && g <= 512 && (g & (g - 1)) == 0;
  const bool pack_ok = !(pl.kind == K_INT && out_fmt == QZ_OUT_PACKED_INT32 && a->num_bits != 4 && a->num_bits != 8);
  const bool al = aligned(w, 16) && aligned(q_out, fq ? 16 : 8) &&
                  (!col_scales || (aligned(col_scales, 16) && cs_ld_batch % 4 == 0));
  if (grp && pow2 && rows_dense && pack_ok && al && batch <= 65535) {
    FastArgs F;
    F.w = (const uint16_t*)w;
    F.n_units = batch * rows * cols / 8;
    F.units_per_batch = rows * cols / 8;
    F.units_per_row = cols / 8;
    F.ld_batch = batch > 1 ? ld_batch : rows * cols;
    F.p = pl.p;
    F.out_fmt = out_fmt;
    F.scale_bytes = pl.scale_bytes;
    F.q_out = q_out;
    F.s_out = s_dst;
    F.zp_out = z_dst;
    F.gscale = gs_dst;
    F.col_scales = col_scales;
    F.cs_ld_batch = cs_ld_batch;
    F.tab = nullptr;
    F.n_tab = 0;
    F.n_seg = 0;
    F.wt_from = 0xffffffffu;  // set with the grid below
    int logl = 0;
    while ((8 << logl) < g) ++logl;
    const bool nt = batch * rows * cols * 2 > (fq ? QZ_NT_BYTES : QZ_NT_BYTES_Q);
    const int64_t fq_yblocks = cdiv(cdiv(rows, FQ_ROWS), FBLOCK / WAVE);
    FqcFn fqc = (fq && col_scales) ? pick_fqc(logl, pl.kind, pl.p.sym != 0, nt) : nullptr;
    if (fqc && fq_yblocks <= 65535) {
      hipLaunchKernelGGL(fqc, dim3((unsigned)cdiv(F.units_per_row, WAVE), (unsigned)fq_yblocks, (unsigned)batch),
                         dim3(FBLOCK), 0, st, F, rows);
      return launch_err();
    }
    const int64_t n_tiles = cdiv(F.units_per_batch, tile_unroll(fq, nt) * WAVE);
    const int64_t blocks = cdiv(n_tiles, FBLOCK / WAVE);
    if (!fq && pl.kind == K_INT && out_fmt == QZ_OUT_PACKED_INT32 && a->num_bits == 4 && F.units_per_batch % 4 == 0 &&
        aligned(q_out, 16))
      F.wt_from = wt_tail_from(blocks * batch, batch * F.units_per_batch * 4);
    hipLaunchKernelGGL(pick_fast(logl, pl.kind, pl.p.sym != 0, fq, nt), dim3((unsigned)blocks, (unsigned)batch),
                       dim3(FBLOCK), 0, st, F);
    return launch_err();
  }

  // FP8_BLOCK 128 x 128 (qz_block.hip): strips of NB blocks per workgroup, 16-B code stores
  if (QZ_BLK_FAST && a->strategy == QZ_BLOCK && pl.kind == K_FP8 && out_fmt == QZ_OUT_FP8 && a->block_h == 128 &&
      a->block_w == 128) {
    BlockFp8Job J{w, batch, rows, cols, ld_row, batch > 1 ? ld_batch : rows * ld_row, q_out, s_dst, nullptr};
    if (block_fp8_ok(J)) return block_fp8_launch(J, pl.p, st);
  }

  // single-pass tile path: BLOCK tiles, CHANNEL rows, wide groups (one workgroup per group)
  {
    int64_t th = 0, tw = 0;
    if (a->strategy == QZ_BLOCK) { th = a->block_h; tw = a->block_w; }
    else if (a->strategy == QZ_CHANNEL) { th = 1; tw = cols; }
    else if (grp && g > 0) { th = 1; tw = g; }
    const int64_t U = th * (tw / 8);
    const bool kind_ok = pl.kind == K_INT || pl.kind == K_FP8 || pl.kind == K_FP4;
    const bool row_al = ld_row % 8 == 0 && (batch == 1 || ld_batch % 8 == 0) && cols % 8 == 0;
    if (!fq && kind_ok && th > 0 && tw % 8 == 0 && U >= 64 && U <= 16 * BLOCK && row_al && pack_ok && al &&
        batch <= 65535) {
      FastArgs F;
      F.w = (const uint16_t*)w;
      F.n_units = batch * rows * cols / 8;
      F.units_per_batch = rows * cols / 8;
      F.units_per_row = cols / 8;
      F.ld_batch = batch > 1 ? ld_batch : rows * ld_row;
      F.p = pl.p;
      F.out_fmt = out_fmt;
      F.scale_bytes = pl.scale_bytes;
      F.q_out = q_out;
      F.s_out = s_dst;
      F.zp_out = z_dst;
      F.gscale = gs_dst;
      F.col_scales = nullptr;
      F.cs_ld_batch = 0;
      F.tab = nullptr;
      F.n_tab = 0;
      F.n_seg = 0;
      F.wt_from = 0xffffffffu;
      TileArgs T;
      T.rows = rows;
      T.tile_rows = th;
      T.tile_w8 = tw / 8;
      T.tiles_c = cols / tw;
      T.ld_row = ld_row;
      const int64_t tiles = (rows / th) * (cols / tw);
      int maxu = 1;
      while (maxu * BLOCK < U) maxu *= 2;
      const bool nt = batch * rows * cols * 2 > QZ_NT_BYTES;
      hipLaunchKernelGGL(pick_tile(pl.kind, pl.p.sym != 0, maxu, nt), dim3((unsigned)tiles, (unsigned)batch), dim3(BLOCK),
                         0, st, F, T);
      return launch_err();
    }
  }

  // generic: min/max -> qparams -> quantize
  if ((rc = run_minmax(G, ng, W.kmin, W.kmax, st))) return rc;
  hipLaunchKernelGGL(k_qparams_keys, dim3((unsigned)cdiv(ng, 256)), dim3(256), 0, st, pl.p, W.kmin, W.kmax, ng,
                     pl.ng_item, (const float*)gs_dst, pl.scale_bytes, s_dst, z_dst);
  if ((rc = launch_err())) return rc;
  int64_t per_item = 1;
  if (out_fmt == QZ_OUT_PACKED_INT32) per_item = 32 / a->num_bits;
  else if (out_fmt == QZ_OUT_FP4_PACKED) per_item = 2;
  const int64_t ipr = cdiv(cols, per_item);
  const int64_t items = batch * rows * ipr;
  hipLaunchKernelGGL(k_quant_generic, dim3((unsigned)cdiv(items, 256)), dim3(256), 0, st, G, pl.p, (int)out_fmt,
                     pl.scale_fmt, (const void*)s_dst, (const int8_t*)z_dst, (const float*)gs_dst, q_out, ipr,
                     per_item);
  return launch_err();
}

int qz_quantize(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row, int64_t ld_batch,
                const qz_args* a, int32_t out_fmt, void* q_out, void* scale_out, int8_t* zp_out, float* gscale_out,
                void* workspace, size_t workspace_bytes, qz_stream_t stream) {
  return quantize_impl(w, batch, rows, cols, ld_row, ld_batch, a, out_fmt, q_out, scale_out, zp_out, gscale_out,
                       nullptr, 0, workspace, workspace_bytes, (hipStream_t)stream);
}

int qz_quantize_many(int64_t n, const void* const* w, void* const* q_out, void* const* scale_out,
                     int8_t* const* zp_out, float* const* gscale_out, int64_t batch, int64_t rows, int64_t cols,
                     int64_t ld_row, int64_t ld_batch, const qz_args* a, int32_t out_fmt, void* workspace,
                     size_t workspace_bytes, qz_stream_t stream) {
  if (n < 0) return QZ_ERR_SHAPE;
  if (n > 0 && (!w || !q_out || !scale_out)) return QZ_ERR_NULL;
  for (int64_t i = 0; i < n; ++i) {  // one launch per weight, in order on the stream
    const int rc = quantize_impl(w[i], batch, rows, cols, ld_row, ld_batch, a, out_fmt, q_out[i], scale_out[i],
                                 zp_out ? zp_out[i] : nullptr, gscale_out ? gscale_out[i] : nullptr, nullptr, 0,
                                 workspace, workspace_bytes, (hipStream_t)stream);
    if (rc) return rc;
  }
  return QZ_OK;
}

int qz_quantize_grouped(int64_t n, const uint64_t* table, int64_t rows, int64_t cols, const qz_args* a,
                        int32_t out_fmt, qz_stream_t stream) {
  if (n == 0) return QZ_OK;
  if (n < 0 || n > 65535 || rows <= 0 || cols <= 0) return QZ_ERR_SHAPE;
  if (!table || !a) return QZ_ERR_NULL;
  Plan pl;
  int rc = make_plan(a, rows, cols, &pl);
  if (rc) return rc;
  if ((rc = check_out_fmt(pl, out_fmt))) return rc;
  if (a->strategy == QZ_BLOCK) {  // FP8_BLOCK 128 x 128: one strip-kernel launch over the table
    if (!QZ_BLK_FAST || pl.kind != K_FP8 || out_fmt != QZ_OUT_FP8 || a->block_h != 128 || a->block_w != 128)
      return QZ_ERR_FORMAT;
    BlockFp8Job J{nullptr, n, rows, cols, cols, rows * cols, nullptr, nullptr, table};
    return block_fp8_ok(J) ? block_fp8_launch(J, pl.p, (hipStream_t)stream) : QZ_ERR_FORMAT;
  }
  const int64_t g = a->group_size;
  const bool grp = a->strategy == QZ_GROUP || a->strategy == QZ_TENSOR_GROUP;
  const bool pow2 = g >= 8 && g <= 512 && (g & (g - 1)) == 0;
  const bool pack_ok = !(pl.kind == K_INT && out_fmt == QZ_OUT_PACKED_INT32 && a->num_bits != 4 && a->num_bits != 8);
  // the single-pass group path only (no per-tensor pre-pass, no fake-quant)
  if (!grp || !pow2 || !pack_ok || pl.kind == K_NV || out_fmt == QZ_OUT_FAKEQUANT || cols % 8) return QZ_ERR_FORMAT;
  if (!aligned(table, 8)) return QZ_ERR_ALIGN;
  FastArgs F;
  F.w = nullptr;
  F.n_units = rows * cols / 8;
  F.units_per_batch = rows * cols / 8;
  F.units_per_row = cols / 8;
  F.ld_batch = rows * cols;
  F.p = pl.p;
  F.out_fmt = out_fmt;
  F.scale_bytes = pl.scale_bytes;
  F.q_out = F.s_out = nullptr;
  F.zp_out = nullptr;
  F.gscale = nullptr;
  F.col_scales = nullptr;
  F.cs_ld_batch = 0;
  F.tab = table;
  F.n_tab = n;
  F.n_seg = 0;
  F.wt_from = 0xffffffffu;
  int logl = 0;
  while ((8 << logl) < g) ++logl;
  const bool nt = n * rows * cols * 2 > QZ_NT_BYTES_Q;
  const int64_t n_tiles = cdiv(F.units_per_batch, tile_unroll(false, nt) * WAVE);
  const int64_t blocks = cdiv(n_tiles, FBLOCK / WAVE);
  if (pl.kind == K_INT && out_fmt == QZ_OUT_PACKED_INT32 && a->num_bits == 4 && F.units_per_batch % 4 == 0)
    F.wt_from = wt_tail_from(blocks * n, n * F.units_per_batch * 4);
  hipLaunchKernelGGL(pick_fast(logl, pl.kind, pl.p.sym != 0, false, nt, true), dim3((unsigned)blocks, (unsigned)n),
                     dim3(FBLOCK), 0, (hipStream_t)stream, F);
  return launch_err();
}

int64_t qz_grouped_blocks(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0 || cols % 8) return -1;
  return cdiv(cdiv(rows * cols / 8, tile_unroll(false, true) * WAVE), FBLOCK / WAVE);
}

int qz_quantize_grouped_var(int64_t n, const uint64_t* table, const int64_t* rows, const int64_t* cols,
                            const qz_args* a, int32_t out_fmt, qz_stream_t stream) {
  if (n == 0) return QZ_OK;
  if (n < 0 || n > 65535) return QZ_ERR_SHAPE;
  if (!table || !rows || !cols || !a) return QZ_ERR_NULL;
  const int64_t g = a->group_size;
  const bool grp = a->strategy == QZ_GROUP || a->strategy == QZ_TENSOR_GROUP;
  const bool pow2 = g >= 8 && g <= 512 && (g & (g - 1)) == 0;
  FastArgs F;
  F.n_seg = 0;
  Plan pl;
  int64_t blocks = 0;
  for (int64_t i = 0; i < n; ++i) {  // every shape validated as qz_quantize_grouped would
    if (rows[i] <= 0 || cols[i] <= 0 || cols[i] % 8) return QZ_ERR_SHAPE;
    int rc = make_plan(a, rows[i], cols[i], &pl);
    if (rc) return rc;
    const bool new_seg = i == 0 || rows[i] != rows[i - 1] || cols[i] != cols[i - 1];
    if (new_seg) {  // runs of equal shapes form the segments
      if (F.n_seg == QZ_MAX_SEG) return QZ_ERR_SHAPE;
      const int sgi = F.n_seg++;
      const int64_t bpw = qz_grouped_blocks(rows[i], cols[i]);
      F.seg_block[sgi] = (uint32_t)blocks;
      F.seg_bpw[sgi] = (uint32_t)bpw;
      F.seg_magic[sgi] = (uint32_t)(0xffffffffull / (uint64_t)bpw);  // q0 >= floor(rel/bpw) - 1
      F.seg_w0[sgi] = (uint32_t)i;
      F.seg_units[sgi] = rows[i] * cols[i] / 8;
    }
    blocks += qz_grouped_blocks(rows[i], cols[i]);
    if (blocks > 0x7fffffffLL) return QZ_ERR_SHAPE;
  }
  F.seg_block[F.n_seg] = (uint32_t)blocks;
  for (int i = F.n_seg; i < QZ_MAX_SEG; ++i) {  // unused entries: never selected
    if (i > F.n_seg) F.seg_block[i] = 0xffffffffu;
    F.seg_bpw[i] = 1; F.seg_magic[i] = 0xffffffffu; F.seg_w0[i] = 0; F.seg_units[i] = 0;
  }
  int rc = check_out_fmt(pl, out_fmt);
  if (rc) return rc;
  const bool pack_ok = !(pl.kind == K_INT && out_fmt == QZ_OUT_PACKED_INT32 && a->num_bits != 4 && a->num_bits != 8);
  if (!grp || !pow2 || !pack_ok || pl.kind == K_NV || out_fmt == QZ_OUT_FAKEQUANT) return QZ_ERR_FORMAT;
  if (!aligned(table, 8)) return QZ_ERR_ALIGN;
  F.w = nullptr;
  F.n_units = 0;
  F.units_per_batch = 0;  // per segment
  F.units_per_row = 0;
  F.ld_batch = 0;
  F.p = pl.p;
  F.out_fmt = out_fmt;
  F.scale_bytes = pl.scale_bytes;
  F.q_out = F.s_out = nullptr;
  F.zp_out = nullptr;
  F.gscale = nullptr;
  F.col_scales = nullptr;
  F.cs_ld_batch = 0;
  F.tab = table;
  F.n_tab = n;
  bool wt_ok = pl.kind == K_INT && out_fmt == QZ_OUT_PACKED_INT32 && a->num_bits == 4;
  int64_t units = 0;
  for (int i = 0; i < n; ++i) units += rows[i] * cols[i] / 8;
  for (int i = 0; i < F.n_seg; ++i) wt_ok = wt_ok && F.seg_units[i] % 4 == 0;
  F.wt_from = wt_ok ? wt_tail_from(blocks, units * 4) : 0xffffffffu;
  int logl = 0;
  while ((8 << logl) < g) ++logl;
  hipLaunchKernelGGL(pick_fast(logl, pl.kind, pl.p.sym != 0, false, true, true), dim3((unsigned)blocks, 1),
                     dim3(FBLOCK), 0, (hipStream_t)stream, F);
  return launch_err();
}

int qz_awq_fake_quant(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row, int64_t ld_batch,
                      const qz_args* a, const float* col_scales, void* w_out, void* workspace, size_t workspace_bytes,
                      qz_stream_t stream) {
  return quantize_impl(w, batch, rows, cols, ld_row, ld_batch, a, QZ_OUT_FAKEQUANT, w_out, nullptr, nullptr, nullptr,
                       col_scales, 0, workspace, workspace_bytes, (hipStream_t)stream);
}

int qz_awq_fake_quant_batched(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row,
                              int64_t ld_batch, const qz_args* a, const float* col_scales, int64_t cs_ld_batch,
                              void* w_out, void* workspace, size_t workspace_bytes, qz_stream_t stream) {
  if (!col_scales) return QZ_ERR_NULL;
  return quantize_impl(w, batch, rows, cols, ld_row, ld_batch, a, QZ_OUT_FAKEQUANT, w_out, nullptr, nullptr, nullptr,
                       col_scales, cs_ld_batch, workspace, workspace_bytes, (hipStream_t)stream);
}

size_t qz_nvfp4_sync_size(int64_t n_slices) {
  return n_slices < 0 ? 0 : 4 * NV_SYNC_STRIDE * (size_t)n_slices;
}

int qz_quantize_nvfp4(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_batch, const qz_args* a,
                      void* q_out, void* scale_out, float* gscale_out, void* sync, size_t sync_bytes,
                      qz_stream_t stream) {
  if (!w || !q_out || !scale_out || !gscale_out) return QZ_ERR_NULL;
  if (batch <= 0 || batch > 0x7fffffff) return QZ_ERR_SHAPE;
  Plan pl;
  int rc = nv_args_ok(a, rows, cols, &pl);
  if (rc) return rc;
  if (batch > 1 && (ld_batch < rows * cols || ld_batch % 8)) return QZ_ERR_SHAPE;
  if (!aligned(w, 16) || !aligned(q_out, 4)) return QZ_ERR_ALIGN;
  NvArgs A;
  A.tab = nullptr;
  A.w = (const uint16_t*)w;
  A.ld_batch = batch > 1 ? ld_batch : rows * cols;
  A.q_out = q_out;
  A.s_out = scale_out;
  A.gs_out = gscale_out;
  A.n_slices = batch;
  A.units_per_slice = rows * cols / 8;
  A.p = pl.p;
  return nv_launch(A, false, sync, sync_bytes, (hipStream_t)stream);
}

int qz_quantize_grouped_nvfp4(int64_t n, const uint64_t* table, int64_t rows, int64_t cols, const qz_args* a,
                              void* sync, size_t sync_bytes, qz_stream_t stream) {
  if (n == 0) return QZ_OK;
  if (n < 0 || n > 0x7fffffff || rows <= 0 || cols <= 0) return QZ_ERR_SHAPE;
  if (!table) return QZ_ERR_NULL;
  if (!aligned(table, 8)) return QZ_ERR_ALIGN;
  Plan pl;
  int rc = nv_args_ok(a, rows, cols, &pl);
  if (rc) return rc;
  NvArgs A;
  A.tab = table;
  A.w = nullptr;
  A.ld_batch = 0;
  A.q_out = A.s_out = nullptr;
  A.gs_out = nullptr;
  A.n_slices = n;
  A.units_per_slice = rows * cols / 8;
  A.p = pl.p;
  return nv_launch(A, true, sync, sync_bytes, (hipStream_t)stream);
}

int qz_quantize_qparams(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row, int64_t ld_batch,
                        const qz_args* a, int32_t out_fmt, const void* scale, const int8_t* zp, const float* gscale,
                        void* q_out, qz_stream_t stream) {
  if (!w || !q_out || !scale || !a) return QZ_ERR_NULL;
  if (batch <= 0) return QZ_ERR_SHAPE;
  Plan pl;
  int rc = make_plan(a, rows, cols, &pl);
  if (rc) return rc;
  if ((rc = check_out_fmt(pl, out_fmt))) return rc;
  if (pl.kind == K_NV && !gscale) return QZ_ERR_NULL;
  if (!pl.p.sym && !zp) return QZ_ERR_NULL;
  if (ld_row < cols || (batch > 1 && ld_batch < rows * ld_row)) return QZ_ERR_SHAPE;
  GenArgs G = gen_args(w, batch, rows, cols, ld_row, ld_batch, a, pl, nullptr);
  int64_t per_item = 1;
  if (out_fmt == QZ_OUT_PACKED_INT32) per_item = 32 / a->num_bits;
  else if (out_fmt == QZ_OUT_FP4_PACKED) per_item = 2;
  const int64_t ipr = cdiv(cols, per_item);
  const int64_t items = batch * rows * ipr;
  hipLaunchKernelGGL(k_quant_generic, dim3((unsigned)cdiv(items, 256)), dim3(256), 0, (hipStream_t)stream, G, pl.p,
                     (int)out_fmt, pl.scale_fmt, scale, zp, gscale, q_out, ipr, per_item);
  return launch_err();
}

int qz_observe_minmax(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row, int64_t ld_batch,
                      const qz_args* a, void* min_out, void* max_out, void* workspace, size_t workspace_bytes,
                      qz_stream_t stream) {
  if (!w || !min_out || !max_out || !a) return QZ_ERR_NULL;
  Plan pl;
  qz_args a2 = *a;
  if (a2.strategy == QZ_TENSOR_GROUP) a2.strategy = QZ_GROUP;
  int rc = make_plan(&a2, rows, cols, &pl);
  if (rc == QZ_ERR_FORMAT) rc = QZ_OK;  // observation does not depend on the format
  if (rc) return rc;
  if (a2.strategy == QZ_TENSOR) pl.ng_item = 1;
  else if (a2.strategy == QZ_CHANNEL) pl.ng_item = rows;
  else if (a2.strategy == QZ_BLOCK) pl.ng_item = (rows / a2.block_h) * (cols / a2.block_w);
  else pl.ng_item = rows * (cols / a2.group_size);
  const int64_t ng = batch * pl.ng_item;
  if (!workspace || workspace_bytes < (size_t)8 * ng) return QZ_ERR_WORKSPACE;
  uint32_t* kmin = (uint32_t*)workspace;
  uint32_t* kmax = kmin + ng;
  GenArgs G = gen_args(w, batch, rows, cols, ld_row, ld_batch, &a2, pl, nullptr);
  if ((rc = run_minmax(G, ng, kmin, kmax, (hipStream_t)stream))) return rc;
  hipLaunchKernelGGL(k_keys_to_bf16, dim3((unsigned)cdiv(ng, 256)), dim3(256), 0, (hipStream_t)stream, kmin, kmax, ng,
                     (uint16_t*)min_out, (uint16_t*)max_out);
  return launch_err();
}

int qz_calculate_qparams(const void* min_vals, const void* max_vals, int64_t n, const qz_args* a,
                         const float* gscale, void* scale_out, int8_t* zp_out, qz_stream_t stream) {
  if (!min_vals || !max_vals || !scale_out || !a) return QZ_ERR_NULL;
  if (n <= 0) return QZ_ERR_SHAPE;
  Plan pl;
  qz_args a2 = *a;
  int rc = make_plan(&a2, 1, a2.group_size > 0 ? a2.group_size : 1, &pl);
  if (rc == QZ_ERR_BLOCK || rc == QZ_ERR_GROUP) rc = QZ_OK;
  if (rc) return rc;
  if (pl.kind == K_NV && !gscale) return QZ_ERR_NULL;
  hipLaunchKernelGGL(k_qparams_bf16, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, pl.p,
                     (const uint16_t*)min_vals, (const uint16_t*)max_vals, n, gscale, pl.scale_bytes, scale_out, zp_out);
  return launch_err();
}

int qz_dequantize(const void* q, int64_t batch, int64_t rows, int64_t cols, const qz_args* a, int32_t in_fmt,
                  const void* scale, const int8_t* zp, const float* gscale, void* w_out, qz_stream_t stream) {
  if (!q || !a || !scale || !w_out) return QZ_ERR_NULL;
  if (batch <= 0) return QZ_ERR_SHAPE;
  Plan pl;
  int rc = make_plan(a, rows, cols, &pl);
  if (rc) return rc;
  if (in_fmt == QZ_OUT_FAKEQUANT || (rc = check_out_fmt(pl, in_fmt))) return rc ? rc : QZ_ERR_FORMAT;
  if (pl.kind == K_NV && !gscale) return QZ_ERR_NULL;
  if (!pl.p.sym && !zp) return QZ_ERR_NULL;
  GenArgs G = gen_args(nullptr, batch, rows, cols, cols, rows * cols, a, pl, nullptr);
  const int64_t n = batch * rows * cols;
  hipLaunchKernelGGL(k_dequant_generic, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, q, batch,
                     rows, cols, pl.p, (int)in_fmt, G, pl.scale_fmt, scale, zp, gscale, (uint16_t*)w_out);
  return launch_err();
}

int qz_pack_int32(const int8_t* v, int64_t rows, int64_t cols, int32_t num_bits, int32_t packed_dim, int32_t* out,
                  qz_stream_t stream) {
  if (!v || !out) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0) return QZ_ERR_SHAPE;
  if (num_bits < 1 || num_bits > 8) return QZ_ERR_BITS;
  if (packed_dim != 0 && packed_dim != 1) return QZ_ERR_FORMAT;
  const int pf = 32 / num_bits;
  const int64_t n = packed_dim == 1 ? rows * cdiv(cols, pf) : cdiv(rows, pf) * cols;
  hipLaunchKernelGGL(k_pack_int32, dim3((unsigned)cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, v, rows, cols,
                     (int)num_bits, (int)packed_dim, out);
  return launch_err();
}

}  // extern "C"
