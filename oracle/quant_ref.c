/*
 * oracle/quant_ref.c -- plain-C restatement of the per-linear weight quantize step.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle/ct_torch.py header).  Linked only by tests/ and the
 * bench's CPU-baseline leg, never by quantizers_amd/.  It restates, with explicit bf16
 * round-to-nearest-even at every point where compressed-tensors materialises a bf16 tensor,
 * the arithmetic SURVEY.md Appendix A describes ([3P] compressed-tensors>=0.13
 * calculate_qparams / _quantize / pack_to_int32 / cast_to_fp4 / pack_fp4_to_uint8, called
 * from scripts/do_oneshot.py:179-197).  It is an independent second implementation of the
 * same algorithm as oracle/ct_torch.py (torch op sequence); tests require the two to agree
 * bit for bit.  Parity against the third-party packages themselves is UNPINNED (absent).
 *
 * Build: make -C oracle   (gcc -O2 -ffp-contract=off; no fast-math: IEEE division/rint).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { ST_TENSOR = 0, ST_CHANNEL = 1, ST_GROUP = 2, ST_BLOCK = 3, ST_TENSOR_GROUP = 4 };
enum { TY_INT = 0, TY_FLOAT = 1 };
enum { SC_NATIVE = 0, SC_FP8 = 2, SC_E8M0 = 3 };

static inline uint32_t fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float ffrom(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static inline float bf2f(uint16_t h) { return ffrom((uint32_t)h << 16); }
static inline uint16_t f2bf(float f) {
  uint32_t u = fbits(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
static inline float bfr(float f) { return bf2f(f2bf(f)); } /* round an f32 result to bf16 */

/* torch.clamp semantics: NaN propagates */
static inline float clampf_t(float x, float lo, float hi) {
  if (isnan(x)) return x;
  return x < lo ? lo : (x > hi ? hi : x);
}

/* float -> float8_e4m3fn, RNE (input already clamped to +-448 in every caller). */
static uint8_t f2e4m3(float f) {
  uint8_t sign = (fbits(f) >> 24) & 0x80;
  if (isnan(f)) return 0x7f | sign;
  float a = fabsf(f);
  if (a < 0.015625f) { /* subnormal: units of 2^-9 */
    float n = nearbyintf(a * 512.0f);
    return sign | (uint8_t)n;
  }
  int e = ilogbf(a);
  float m = ldexpf(a, -e);            /* [1,2) exact */
  float t = nearbyintf((m - 1.0f) * 8.0f);
  if (t == 8.0f) { e += 1; t = 0.0f; }
  return sign | (uint8_t)(((e + 7) << 3) | (int)t);
}
static float e4m32f(uint8_t c) {
  float s = (c & 0x80) ? -1.f : 1.f;
  int e = (c >> 3) & 0xf, m = c & 7;
  if (e == 15 && m == 7) return NAN;
  if (e == 0) return s * ldexpf((float)m, -9);
  return s * ldexpf(1.0f + m / 8.0f, e - 7);
}

/* FP4_E2M1_DATA.cast_to_fp4 thresholds, applied to |x|; returns the grid index, sign bit
 * = signbit of sign(x)*|q| (torch.sign(0) = 0 so zero stays +0, small negatives give -0). */
static uint8_t fp4_code(float x) {
  if (x != x) return 0; /* D17: a NaN quotient (0 / 0 under an overflowed NVFP4 global scale) */
  float a = fabsf(x);
  int idx;
  if (a <= 0.25f) idx = 0;
  else if (a < 0.75f) idx = 1;
  else if (a <= 1.25f) idx = 2;
  else if (a < 1.75f) idx = 3;
  else if (a <= 2.5f) idx = 4;
  else if (a < 3.5f) idx = 5;
  else if (a <= 5.0f) idx = 6;
  else idx = 7;
  int neg = (x < 0.0f); /* sign(x) = -1 -> result carries the sign bit even when |q| = 0 */
  return (uint8_t)(idx | (neg << 3));
}

typedef struct {
  int num_bits, type, symmetric, strategy, group_size, block_h, block_w, scale_fmt;
} qref_args;

/* number of groups and per-element group id */
static int64_t n_groups(const qref_args* a, int64_t R, int64_t C) {
  switch (a->strategy) {
    case ST_TENSOR: return 1;
    case ST_CHANNEL: return R;
    case ST_GROUP: case ST_TENSOR_GROUP: return R * (C / a->group_size);
    case ST_BLOCK: return (R / a->block_h) * (C / a->block_w);
  }
  return -1;
}
static inline int64_t gid(const qref_args* a, int64_t C, int64_t r, int64_t c) {
  switch (a->strategy) {
    case ST_TENSOR: return 0;
    case ST_CHANNEL: return r;
    case ST_GROUP: case ST_TENSOR_GROUP: return r * (C / a->group_size) + c / a->group_size;
    default: return (r / a->block_h) * (C / a->block_w) + c / a->block_w;
  }
}

/*
 * qref_quantize: observe (memoryless min/max) -> calculate_qparams -> quantize.
 * Outputs: q[R*C] as int8 (int) / e4m3 bytes (fp8) / fp4 codes 0..15 (fp4), unpacked;
 * scale_bits[ng] as uint16 bf16 (native) / uint8 (fp8 or e8m0) in a uint16 slot;
 * zp[ng] int8; gscale[0] f32 for tensor_group.
 */
int qref_quantize(const uint16_t* w, int64_t R, int64_t C, const qref_args* a,
                  uint8_t* q, uint16_t* scale_bits, int8_t* zp, float* gscale) {
  int64_t ng = n_groups(a, R, C);
  if (ng <= 0) return -1;
  float* mn = (float*)malloc(sizeof(float) * ng);
  float* mx = (float*)malloc(sizeof(float) * ng);
  float* sc = (float*)malloc(sizeof(float) * ng); /* effective divisor per group */
  for (int64_t i = 0; i < ng; ++i) { mn[i] = INFINITY; mx[i] = -INFINITY; }
  float tmn = INFINITY, tmx = -INFINITY;
  for (int64_t r = 0; r < R; ++r)
    for (int64_t c = 0; c < C; ++c) {
      float v = bf2f(w[r * C + c]);
      int64_t g = gid(a, C, r, c);
      if (v < mn[g]) mn[g] = v;
      if (v > mx[g]) mx[g] = v;
      if (v < tmn) tmn = v;
      if (v > tmx) tmx = v;
    }
  float qmin, qmax;
  if (a->type == TY_INT) { qmin = -ldexpf(1.f, a->num_bits - 1); qmax = ldexpf(1.f, a->num_bits - 1) - 1.f; }
  else if (a->num_bits == 8) { qmin = -448.f; qmax = 448.f; }
  else { qmin = -6.f; qmax = 6.f; }
  float gs = 0.f;
  if (a->strategy == ST_TENSOR_GROUP) {
    /* generate_gparam: (448*6) / absmax in bf16; python-scalar / tensor == reciprocal * scalar */
    float tmin = fminf(tmn, 0.f), tmax = fmaxf(tmx, 0.f);
    float am = fmaxf(fabsf(tmin), fabsf(tmax));
    float rc = bfr(1.0f / am);
    gs = bfr(rc * 2688.0f);
    gscale[0] = gs;
  }
  for (int64_t g = 0; g < ng; ++g) {
    float lo = fminf(mn[g], 0.f), hi = fmaxf(mx[g], 0.f);
    float s, z = 0.f;
    if (a->symmetric) {
      float am = fmaxf(fabsf(lo), fabsf(hi));
      if (a->scale_fmt == SC_E8M0) {
        /* round_to_power_2 (bf16 bit trick) -> exponent field E -> byte = E - 2 */
        uint16_t b = f2bf(am);
        uint16_t p = (uint16_t)(((uint32_t)b + 0x40u) & 0xFF80u);
        int e = (p >> 7) & 0xFF;
        int byte = e - 2; if (byte < 0) byte = 0; if (byte > 254) byte = 254;
        scale_bits[g] = (uint16_t)byte;
        sc[g] = ldexpf(1.0f, byte - 127); /* dense bf16 scale 2^(e-127) (always representable) */
        zp[g] = 0;
        continue;
      }
      s = bfr(am / ((qmax - qmin) / 2.0f));
    } else {
      s = bfr(bfr(hi - lo) / (qmax - qmin));
      float t = bfr(lo / s);
      z = clampf_t(bfr(qmin - t), qmin, qmax);
    }
    if (a->strategy == ST_TENSOR_GROUP) {
      float s32 = gs * s;                                /* f32 * bf16 -> f32 */
      uint8_t s8 = f2e4m3(clampf_t(s32, -448.f, 448.f)); /* round to scale dtype */
      float sf = e4m32f(s8);
      if (sf == 0.f) { s8 = f2e4m3(0.125f); sf = 0.125f; }
      scale_bits[g] = s8;
      sc[g] = sf / gs; /* _quantize: scale / global_scale in f32 */
    } else {
      if (s == 0.f) s = 0.0078125f; /* D1 */
      scale_bits[g] = f2bf(s);
      sc[g] = s;
    }
    zp[g] = isnan(z) ? 0 : (int8_t)nearbyintf(z); /* D10 */
  }
  for (int64_t r = 0; r < R; ++r)
    for (int64_t c = 0; c < C; ++c) {
      int64_t g = gid(a, C, r, c);
      float x = bf2f(w[r * C + c]);
      if (a->type == TY_INT) {
        float t = bfr(x / sc[g]);
        t = bfr(t + (float)zp[g]);
        t = clampf_t(t, qmin, qmax);
        float rq = nearbyintf(t);
        q[r * C + c] = (uint8_t)(int8_t)(isnan(rq) ? 0 : (int)rq);
      } else if (a->num_bits == 8) {
        float t = bfr(x / sc[g]);
        q[r * C + c] = f2e4m3(clampf_t(t, -448.f, 448.f));
      } else {
        float t = (a->strategy == ST_TENSOR_GROUP) ? (x / sc[g]) /* f32 quotient (D5) */
                                                   : bfr(x / sc[g]);
        q[r * C + c] = fp4_code(clampf_t(t, -6.f, 6.f));
      }
    }
  free(mn); free(mx); free(sc);
  return 0;
}

/* pack_to_int32 along dim 1 (cols) of an int8 [R, C] tensor; out int32 [R, ceil(C/pf)] */
void qref_pack_int32(const int8_t* v, int64_t R, int64_t C, int bits, int32_t* out) {
  int pf = 32 / bits;
  int64_t W = (C + pf - 1) / pf;
  uint32_t mask = (1u << bits) - 1u;
  for (int64_t r = 0; r < R; ++r)
    for (int64_t j = 0; j < W; ++j) {
      uint32_t word = 0;
      for (int i = 0; i < pf; ++i) {
        int64_t c = j * pf + i;
        uint32_t u = c < C ? ((uint32_t)(v[r * C + c] + (1 << (bits - 1))) & mask) : 0u;
        word |= u << (bits * i);
      }
      out[r * W + j] = (int32_t)word;
    }
}

/* pack_to_int32(packed_dim=0): pack rows; out int32 [ceil(R/pf), C] */
void qref_pack_int32_dim0(const int8_t* v, int64_t R, int64_t C, int bits, int32_t* out) {
  int pf = 32 / bits;
  int64_t H = (R + pf - 1) / pf;
  uint32_t mask = (1u << bits) - 1u;
  for (int64_t j = 0; j < H; ++j)
    for (int64_t c = 0; c < C; ++c) {
      uint32_t word = 0;
      for (int i = 0; i < pf; ++i) {
        int64_t r = j * pf + i;
        uint32_t u = r < R ? ((uint32_t)(v[r * C + c] + (1 << (bits - 1))) & mask) : 0u;
        word |= u << (bits * i);
      }
      out[j * C + c] = (int32_t)word;
    }
}

/* pack_fp4_to_uint8: element 2k -> low nibble */
void qref_pack_fp4(const uint8_t* codes, int64_t n, uint8_t* out) {
  for (int64_t k = 0; k < n / 2; ++k) out[k] = (uint8_t)((codes[2 * k] & 15) | ((codes[2 * k + 1] & 15) << 4));
}

/* Fused int quant + pack for the bench's CPU leg (same arithmetic as qref_quantize, one pass
 * per group, no heap traffic beyond the outputs): symmetric int, strategy=group. */
int qref_int_sym_group_pack(const uint16_t* w, int64_t R, int64_t C, int bits, int g,
                            int32_t* packed, uint16_t* scale) {
  if (C % g || g % (32 / bits)) return -1;
  float qmax = ldexpf(1.f, bits - 1) - 1.f, qmin = -ldexpf(1.f, bits - 1);
  float half = (qmax - qmin) / 2.0f;
  int pf = 32 / bits;
  uint32_t mask = (1u << bits) - 1u;
  int64_t W = C / pf, G = C / g;
  for (int64_t r = 0; r < R; ++r)
    for (int64_t gi = 0; gi < G; ++gi) {
      const uint16_t* p = w + r * C + gi * g;
      uint16_t am = 0;
      for (int i = 0; i < g; ++i) { uint16_t b = p[i] & 0x7fff; if (b > am) am = b; }
      float s = bfr(bf2f(am) / half);
      if (s == 0.f) s = 0.0078125f;
      scale[r * G + gi] = f2bf(s);
      for (int j = 0; j < g / pf; ++j) {
        uint32_t word = 0;
        for (int i = 0; i < pf; ++i) {
          float t = clampf_t(bfr(bf2f(p[j * pf + i]) / s), qmin, qmax);
          int qi = (int)nearbyintf(t);
          word |= ((uint32_t)(qi - (int)qmin) & mask) << (bits * i);
        }
        packed[r * W + (gi * g) / pf + j] = (int32_t)word;
      }
    }
  return 0;
}
