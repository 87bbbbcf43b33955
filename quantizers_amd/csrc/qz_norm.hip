// qz_norm.hip -- the model's RMSNorm over 128-wide rows in the model's own arithmetic (gfx950).
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

}  // extern "C"
