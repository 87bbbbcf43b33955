// qz_norm.hip -- the attention block's per-head elementwise steps in the model's own arithmetic
// (gfx950): the 128-wide q / k RMSNorm (qz_rmsnorm128) and the rotary embedding
// (qz_rotary128).
//
// transformers' Qwen3RMSNorm (the q / k head norms of every attention forward; pinned 4.57 by the
// reference) is a chain of PyTorch kernels with f32 intermediates: x.to(f32); pow(2); mean(-1);
// + eps; rsqrt; x * r; .to(bf16); weight * y.  qz_rmsnorm128 does it in one pass, reproducing
// every rounding and PyTorch's summation order (established on the GPU by
// scripts/rmsnorm_probe.py, profiles/r03t_rmsnorm_probe.log):
//   * PyTorch's reduce kernel for a contiguous 128-wide row vectorises the input: 32 threads per
//     row, thread t sums its four squares ((x[4t]^2 + x[4t+1]^2) + x[4t+2]^2) + x[4t+3]^2 (one
//     accumulator per vector lane, combined in order), then a shuffle-down tree with offsets
//     1, 2, 4, 8, 16 -- every other candidate tree differs in about a third of the rows;
//   * the mean is that sum times 1/128 (exact); torch.rsqrt is correctly rounded (it equals
//     f32(1 / sqrt(f64(v))) on every tested value; v_rsq_f32 and rsqrtf differ in ~5 % of rows);
//   * y = bf16(x * r), out = bf16(weight * y).
// Layout: one wave covers two rows (lanes 0-31 and 32-63), each lane 4 consecutive elements (one
// 8-B load and store), so the tree is PyTorch's thread mapping exactly.
#include <hip/hip_runtime.h>

#include "qz_device.h"

using namespace qz;

namespace {

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline bool aligned(const void* p, size_t n) { return ((uintptr_t)p % n) == 0; }
int launch_err() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QZ_OK : (int)e;
}

constexpr int NB_WAVES = 4;  // waves per workgroup: 8 rows

__global__ __launch_bounds__(NB_WAVES * 64) void k_rmsnorm128(const uint16_t* __restrict__ x, int64_t rows,
                                                              int64_t ld, const uint16_t* __restrict__ w, float eps,
                                                              uint16_t* __restrict__ out) {
  const int lane = threadIdx.x & 63, hl = lane & 31;
  const int64_t r = ((int64_t)blockIdx.x * NB_WAVES + (threadIdx.x >> 6)) * 2 + (lane >> 5);
  const bool ok = r < rows;
  const int64_t rr = ok ? r : rows - 1;  // every lane joins the shuffles; loads clamped in bounds
  const uint2 q = *(const uint2*)(x + rr * ld + 4 * hl);
  const float e0 = __uint_as_float(q.x << 16), e1 = __uint_as_float(q.x & 0xffff0000u);
  const float e2 = __uint_as_float(q.y << 16), e3 = __uint_as_float(q.y & 0xffff0000u);
  float v = __fadd_rn(__fadd_rn(__fadd_rn(__fmul_rn(e0, e0), __fmul_rn(e1, e1)), __fmul_rn(e2, e2)), __fmul_rn(e3, e3));
#pragma unroll
  for (int off = 1; off < 32; off <<= 1) v = __fadd_rn(v, __shfl_down(v, off, 64));  // lane 0 / 32: its row
  v = __shfl(v, lane & 32, 64);
  const float var = __fmul_rn(v, 0.0078125f);  // mean: sum * (1 / 128), exact
  const float rs = (float)(1.0 / sqrt((double)__fadd_rn(var, eps)));  // torch.rsqrt: correctly rounded
  const uint2 wq = *(const uint2*)(w + 4 * hl);
  const float y0 = bfr(__fmul_rn(e0, rs)), y1 = bfr(__fmul_rn(e1, rs));
  const float y2 = bfr(__fmul_rn(e2, rs)), y3 = bfr(__fmul_rn(e3, rs));
  uint2 o;
  o.x = (uint32_t)f2bf(__fmul_rn(__uint_as_float(wq.x << 16), y0)) |
        ((uint32_t)f2bf(__fmul_rn(__uint_as_float(wq.x & 0xffff0000u), y1)) << 16);
  o.y = (uint32_t)f2bf(__fmul_rn(__uint_as_float(wq.y << 16), y2)) |
        ((uint32_t)f2bf(__fmul_rn(__uint_as_float(wq.y & 0xffff0000u), y3)) << 16);
  if (ok) *(uint2*)(out + r * 128 + 4 * hl) = o;
}

// Rotary embedding of 128-wide heads (transformers 4.57 apply_rotary_pos_emb with rotate_half):
// out = bf16(bf16(x * cos) + bf16(rotate_half(x) * sin)), rotate_half(x) = cat(-x[64:], x[:64]);
// every product and the sum rounded to bf16 like the three PyTorch kernels (mul, mul, add) the
// composition runs (the negation is exact).  x is [B, H, T, 128] at any B / H / T strides (the
// transposed projection output), cos / sin [B, T, 128] broadcast over H, out at its own strides.
// A lane covers 4 consecutive elements of each half: 16 lanes per row, 4 rows per wave.
__device__ __forceinline__ void ld4(const uint16_t* p, float (&v)[4]) {
  const uint2 q = *(const uint2*)p;
  v[0] = __uint_as_float(q.x << 16);
  v[1] = __uint_as_float(q.x & 0xffff0000u);
  v[2] = __uint_as_float(q.y << 16);
  v[3] = __uint_as_float(q.y & 0xffff0000u);
}
__device__ __forceinline__ void st4(uint16_t* p, const float (&v)[4]) {
  uint2 q;
  q.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  q.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *(uint2*)p = q;
}

__global__ __launch_bounds__(256) void k_rotary128(const uint16_t* __restrict__ x, int64_t xb, int64_t xh, int64_t xt,
                                                   const uint16_t* __restrict__ cs, const uint16_t* __restrict__ sn,
                                                   int64_t cb, int64_t ct, int64_t B, int64_t H, int64_t T,
                                                   uint16_t* __restrict__ out, int64_t ob, int64_t oh, int64_t ot) {
  const int64_t row = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;  // (b, h, t)
  const int l = threadIdx.x & 15;
  if (row >= B * H * T) return;
  const int64_t t = row % T, bh = row / T, h = bh % H, b = bh / H;
  const uint16_t* xr = x + b * xb + h * xh + t * xt;
  const int64_t c0 = b * cb + t * ct;
  float x1[4], x2[4], c1[4], c2[4], s1[4], s2[4], o1[4], o2[4];
  ld4(xr + 4 * l, x1);
  ld4(xr + 64 + 4 * l, x2);
  ld4(cs + c0 + 4 * l, c1);
  ld4(cs + c0 + 64 + 4 * l, c2);
  ld4(sn + c0 + 4 * l, s1);
  ld4(sn + c0 + 64 + 4 * l, s2);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o1[i] = __fadd_rn(bfr(__fmul_rn(x1[i], c1[i])), bfr(__fmul_rn(-x2[i], s1[i])));
    o2[i] = __fadd_rn(bfr(__fmul_rn(x2[i], c2[i])), bfr(__fmul_rn(x1[i], s2[i])));
  }
  uint16_t* orow = out + b * ob + h * oh + t * ot;
  st4(orow + 4 * l, o1);
  st4(orow + 64 + 4 * l, o2);
}

}  // namespace

extern "C" {

int qz_rmsnorm128(const void* x, int64_t rows, int64_t ld, const void* weight, float eps, void* out,
                  qz_stream_t stream) {
  if (rows < 0 || ld < 128) return QZ_ERR_SHAPE;
  if (rows == 0) return QZ_OK;
  if (!x || !weight || !out) return QZ_ERR_NULL;
  if (ld % 4 || !aligned(x, 8) || !aligned(weight, 8) || !aligned(out, 8)) return QZ_ERR_ALIGN;
  const int64_t blocks = cdiv(rows, 2 * NB_WAVES);
  if (blocks > 0x7fffffffLL) return QZ_ERR_SHAPE;
  hipLaunchKernelGGL(k_rmsnorm128, dim3((unsigned)blocks), dim3(NB_WAVES * 64), 0, (hipStream_t)stream,
                     (const uint16_t*)x, rows, ld, (const uint16_t*)weight, eps, (uint16_t*)out);
  return launch_err();
}

int qz_rotary128(const void* x, int64_t B, int64_t H, int64_t T, int64_t xb, int64_t xh, int64_t xt, const void* cos,
                 const void* sin, int64_t cb, int64_t ct, void* out, int64_t ob, int64_t oh, int64_t ot,
                 qz_stream_t stream) {
  if (B < 0 || H < 0 || T < 0) return QZ_ERR_SHAPE;
  if (B == 0 || H == 0 || T == 0) return QZ_OK;
  if (!x || !cos || !sin || !out) return QZ_ERR_NULL;
  for (int64_t s : {xb, xh, xt, cb, ct, ob, oh, ot})
    if (s % 4) return QZ_ERR_ALIGN;
  if (!aligned(x, 8) || !aligned(cos, 8) || !aligned(sin, 8) || !aligned(out, 8)) return QZ_ERR_ALIGN;
  const int64_t blocks = cdiv(B * H * T, 16);  // 16 rows per 256-thread workgroup
  if (blocks > 0x7fffffffLL) return QZ_ERR_SHAPE;
  hipLaunchKernelGGL(k_rotary128, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, (const uint16_t*)x, xb,
                     xh, xt, (const uint16_t*)cos, (const uint16_t*)sin, cb, ct, B, H, T, (uint16_t*)out, ob, oh, ot);
  return launch_err();
}

}  // extern "C"
