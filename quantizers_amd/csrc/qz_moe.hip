// qz_moe.hip -- the tail of a fused-experts MoE forward in the eager arithmetic (gfx950).
//
// transformers' eager experts loop (pinned 4.57 by the reference; moe_eager.py, decision D15)
// ends every routed expert with `current * top_k_weights[token, slot]` (bf16 product) and an
// `index_add_` into a bf16 accumulator, experts in ascending id: each token sums its top-k
// weighted contributions left to right with a bf16 rounding after every add, starting from a
// +0 accumulator.  Composed from PyTorch ops that tail is a weighting pass, a row gather and k
// strided adds over [tokens, hidden] -- ~7 passes over the expert outputs.  qz_moe_combine does
// it in one: per token, read its k expert-sorted output rows in ascending expert order, weight
// and add in registers with the same roundings, write the token row once.  qz_silu_mul /
// qz_moe_silu_mul fuse the `act_fn(gate) * up` between the gate/up and down projections (two
// passes) into one, for dense MLPs and experts alike.
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

template <bool WF32>
__device__ __forceinline__ float route_weight(const void* w, int64_t i) {
  return WF32 ? ((const float*)w)[i] : bf2f(((const uint16_t*)w)[i]);
}

// One workgroup per (token, 2048-column block); lane = 8 columns (one 16-B load per expert row).
// The token's k source rows and weights are workgroup-uniform (scalar loads).
constexpr int CB_THREADS = 256, CB_COLS = CB_THREADS * 8;

template <bool WF32>
__global__ __launch_bounds__(CB_THREADS) void k_moe_combine_v8(const uint16_t* __restrict__ d, const void* w,
                                                                const int64_t* __restrict__ perm,
                                                                const int64_t* __restrict__ src, int64_t H, int k,
                                                                int64_t ncb, uint16_t* __restrict__ out) {
  const int64_t t = blockIdx.x / ncb;
  const int64_t c0 = (blockIdx.x % ncb) * CB_COLS + (int64_t)threadIdx.x * 8;
  if (c0 >= H) return;
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) acc[i] = 0.0f;  // torch.zeros_like: +0
  const int64_t* s = src + t * k;
  for (int j = 0; j < k; ++j) {
    const int64_t r = s[j];
    const float wr = route_weight<WF32>(w, perm[r]);
    const uint4 v = *(const uint4*)(d + r * H + c0);
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x0 = bfr(__uint_as_float(u[q] << 16) * wr);          // bf16 product
      const float x1 = bfr(__uint_as_float(u[q] & 0xffff0000u) * wr);
      acc[2 * q] = bfr(acc[2 * q] + x0);                                 // bf16 accumulator
      acc[2 * q + 1] = bfr(acc[2 * q + 1] + x1);
    }
  }
  uint4 o;
  o.x = (uint32_t)f2bf(acc[0]) | ((uint32_t)f2bf(acc[1]) << 16);
  o.y = (uint32_t)f2bf(acc[2]) | ((uint32_t)f2bf(acc[3]) << 16);
  o.z = (uint32_t)f2bf(acc[4]) | ((uint32_t)f2bf(acc[5]) << 16);
  o.w = (uint32_t)f2bf(acc[6]) | ((uint32_t)f2bf(acc[7]) << 16);
  *(uint4*)(out + t * H + c0) = o;
}

// Any hidden size / alignment: one column per thread.
template <bool WF32>
__global__ __launch_bounds__(CB_THREADS) void k_moe_combine_v1(const uint16_t* __restrict__ d, const void* w,
                                                                const int64_t* __restrict__ perm,
                                                                const int64_t* __restrict__ src, int64_t H, int k,
                                                                int64_t ncb, uint16_t* __restrict__ out) {
  const int64_t t = blockIdx.x / ncb;
  const int64_t c = (blockIdx.x % ncb) * CB_THREADS + threadIdx.x;
  if (c >= H) return;
  float acc = 0.0f;
  const int64_t* s = src + t * k;
  for (int j = 0; j < k; ++j) {
    const int64_t r = s[j];
    acc = bfr(acc + bfr(bf2f(d[r * H + c]) * route_weight<WF32>(w, perm[r])));
  }
  out[t * H + c] = f2bf(acc);
}

// silu(gate) * up: torch's silu kernel (x / (1 + exp(-x)) in f32, rounded to bf16) then the bf16
// product; gate and up are [rows, inter] with their own row strides (the two halves of one fused
// gate/up GEMM output, or two separate projections), out is dense [rows, inter].
__device__ __forceinline__ float silu_bf16(float x) { return bfr(x / (1.0f + expf(-x))); }

__global__ __launch_bounds__(256) void k_silu_mul_v8(const uint16_t* __restrict__ gate, int64_t ldg,
                                                     const uint16_t* __restrict__ up, int64_t ldu, int64_t rows,
                                                     int64_t inter, uint16_t* __restrict__ h) {
  const int64_t per_row = inter / 8;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * per_row) return;
  const int64_t r = i / per_row, c = (i % per_row) * 8;
  const uint4 g = *(const uint4*)(gate + r * ldg + c);
  const uint4 u = *(const uint4*)(up + r * ldu + c);
  const uint32_t ga[4] = {g.x, g.y, g.z, g.w}, ua[4] = {u.x, u.y, u.z, u.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float lo = silu_bf16(__uint_as_float(ga[q] << 16)) * __uint_as_float(ua[q] << 16);
    const float hi = silu_bf16(__uint_as_float(ga[q] & 0xffff0000u)) * __uint_as_float(ua[q] & 0xffff0000u);
    o[q] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
  }
  *(uint4*)(h + r * inter + c) = make_uint4(o[0], o[1], o[2], o[3]);
}

__global__ __launch_bounds__(256) void k_silu_mul_v1(const uint16_t* __restrict__ gate, int64_t ldg,
                                                     const uint16_t* __restrict__ up, int64_t ldu, int64_t rows,
                                                     int64_t inter, uint16_t* __restrict__ h) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= rows * inter) return;
  const int64_t r = i / inter, c = i % inter;
  h[r * inter + c] = f2bf(silu_bf16(bf2f(gate[r * ldg + c])) * bf2f(up[r * ldu + c]));
}

}  // namespace

extern "C" {

int qz_moe_combine(const void* expert_out, int64_t rows, int64_t hidden, const void* weights, int32_t weights_f32,
                   const int64_t* perm, const int64_t* src, int64_t tokens, int32_t top_k, void* out,
                   qz_stream_t stream) {
  if (tokens < 0 || hidden <= 0 || top_k <= 0 || rows != tokens * top_k) return QZ_ERR_SHAPE;
  if (tokens == 0) return QZ_OK;
  if (!out || !expert_out || !weights || !perm || !src) return QZ_ERR_NULL;
  hipStream_t st = (hipStream_t)stream;
  const bool v8 = hidden % 8 == 0 && aligned(expert_out, 16) && aligned(out, 16);
  const int64_t ncb = cdiv(hidden, v8 ? CB_COLS : CB_THREADS);
  if (tokens * ncb > 0x7fffffffLL) return QZ_ERR_SHAPE;
  const dim3 grid((unsigned)(tokens * ncb)), block(CB_THREADS);
  const uint16_t* d = (const uint16_t*)expert_out;
  uint16_t* o = (uint16_t*)out;
  if (v8) {
    if (weights_f32)
      hipLaunchKernelGGL(k_moe_combine_v8<true>, grid, block, 0, st, d, weights, perm, src, hidden, top_k, ncb, o);
    else
      hipLaunchKernelGGL(k_moe_combine_v8<false>, grid, block, 0, st, d, weights, perm, src, hidden, top_k, ncb, o);
  } else {
    if (weights_f32)
      hipLaunchKernelGGL(k_moe_combine_v1<true>, grid, block, 0, st, d, weights, perm, src, hidden, top_k, ncb, o);
    else
      hipLaunchKernelGGL(k_moe_combine_v1<false>, grid, block, 0, st, d, weights, perm, src, hidden, top_k, ncb, o);
  }
  return launch_err();
}

int qz_silu_mul(const void* gate, int64_t ld_gate, const void* up, int64_t ld_up, int64_t rows, int64_t inter,
                void* out, qz_stream_t stream) {
  if (rows < 0 || inter <= 0 || ld_gate < inter || ld_up < inter) return QZ_ERR_SHAPE;
  if (rows == 0) return QZ_OK;
  if (!gate || !up || !out) return QZ_ERR_NULL;
  const bool v8 = inter % 8 == 0 && ld_gate % 8 == 0 && ld_up % 8 == 0 && aligned(gate, 16) && aligned(up, 16) &&
                  aligned(out, 16);
  const int64_t n = v8 ? rows * (inter / 8) : rows * inter;
  if (cdiv(n, 256) > 0x7fffffffLL) return QZ_ERR_SHAPE;
  const dim3 grid((unsigned)cdiv(n, 256)), block(256);
  if (v8)
    hipLaunchKernelGGL(k_silu_mul_v8, grid, block, 0, (hipStream_t)stream, (const uint16_t*)gate, ld_gate,
                       (const uint16_t*)up, ld_up, rows, inter, (uint16_t*)out);
  else
    hipLaunchKernelGGL(k_silu_mul_v1, grid, block, 0, (hipStream_t)stream, (const uint16_t*)gate, ld_gate,
                       (const uint16_t*)up, ld_up, rows, inter, (uint16_t*)out);
  return launch_err();
}

int qz_moe_silu_mul(const void* gate_up, int64_t rows, int64_t inter, int64_t ld, void* out, qz_stream_t stream) {
  if (rows < 0 || inter <= 0 || ld < 2 * inter) return QZ_ERR_SHAPE;
  if (rows == 0) return QZ_OK;
  if (!gate_up) return QZ_ERR_NULL;
  return qz_silu_mul(gate_up, ld, (const uint16_t*)gate_up + inter, ld, rows, inter, out, stream);
}

}  // extern "C"
