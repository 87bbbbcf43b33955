// qz_awq.hip -- AWQ statistics, grid-scale and smoothing kernels (gfx950).
//
// Replaces the elementwise/reduction parts of [3P] llmcompressor AWQModifier (SURVEY.md §8a
// a3, a4, a5 scale computation, a6): the per-channel mean|x| hook, the per-channel mean of
// group-normalised |W| (w_mean), the grid's scale vector and _apply_smoothing.  The
// fake-quant step of the grid search lives in qz_quant.hip (qz_awq_fake_quant); the parent
// forwards are PyTorch GEMMs on the host side.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "qz_device.h"

using namespace qz;

namespace {

constexpr int WAVE = 64;
typedef uint32_t qz_u32x4 __attribute__((ext_vector_type(4)));

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
__device__ __forceinline__ int64_t cdiv_d(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline bool aligned(const void* p, size_t n) { return ((uintptr_t)p % n) == 0; }
int launch_err() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? QZ_OK : (int)e;
}

// ---------------------------------------------------------- a3: sum_t |x[t, c]|
// Both statistics reduce a tall [rows, C] bf16 matrix into per-column sums with the same stage-1
// shape: a workgroup of SWP waves covers one 512-column window (lane = 8 columns, one 16-B load
// per row) x a chunk of rows; wave w takes rows w, w + SWP, ... in order, SNB rows per batch, and
// the next batch's loads are issued before the current batch is summed (software pipelined: a
// wave always has SNB 16-B loads in flight while it computes).  Load addresses are clamped into
// the matrix so no load is predicated (the compiler can then count vmcnt instead of draining);
// rows past the chunk end are skipped by a wave-uniform branch.  The SWP wave sums are added in a
// fixed order (((s0 + s1) + s2) + ...) through LDS -> part[chunk][c]; stage 2 (k_colsum_final)
// adds the chunks in a fixed order: deterministic.
constexpr int QZ_ABSMEAN_WPB = 8; // waves per absmean stage-1 workgroup
constexpr int QZ_WMEAN_WPB = 8; // waves per w_mean stage-1 workgroup
constexpr int QZ_ABSMEAN_NB = 8; // activation rows per batch (loads in flight per lane)
constexpr int QZ_WMEAN_NB = 4; // weight rows per batch (f64 sums: fewer, to keep VGPRs < 128)
constexpr int AWP = QZ_ABSMEAN_WPB, WWP = QZ_WMEAN_WPB;

// walk rows r0 + wv, r0 + wv + SWP, ... < r1 of the 8 columns at col (clamped into [0, C - 8]);
// f(v) is called once per row in row order
template <int SWP, int SNB, typename F>
__device__ __forceinline__ void stats_rows(const uint16_t* base, int64_t ld, int64_t r0, int64_t r1, int wv, F&& f) {
  // row offsets in 32 x 32 -> 64-bit products (one v_mad_u64_u32; the host guarantees rows and
  // ld < 2^31)
  const uint32_t rlast = (uint32_t)(r1 - 1), uld = (uint32_t)ld;
  auto ld16 = [&](int64_t r) {
    return *reinterpret_cast<const uint4*>(base + (uint64_t)std::min((uint32_t)r, rlast) * uld);
  };
  int64_t r = r0 + wv;
  if (r >= r1) return;
  uint4 cur[SNB];
#pragma unroll
  for (int j = 0; j < SNB; ++j) cur[j] = ld16(r + (int64_t)j * SWP);
  // in the loop the next batch starts inside the chunk, so every row of the current one is valid
  for (; r + (int64_t)SNB * SWP < r1; r += (int64_t)SNB * SWP) {
    uint4 nxt[SNB];
#pragma unroll
    for (int j = 0; j < SNB; ++j) nxt[j] = ld16(r + (int64_t)(SNB + j) * SWP);
#pragma unroll
    for (int j = 0; j < SNB; ++j) f(cur[j]);
#pragma unroll
    for (int j = 0; j < SNB; ++j) cur[j] = nxt[j];
  }
#pragma unroll
  for (int j = 0; j < SNB; ++j)
    if (r + (int64_t)j * SWP < r1) f(cur[j]);
}

template <int SWP, typename T>
__device__ __forceinline__ void stats_block_sum(T (*red)[512], const T* acc, int lane, int wv, int64_t C, T* dst) {
#pragma unroll
  for (int i = 0; i < 8; ++i) red[wv][lane * 8 + i] = acc[i];
  __syncthreads();
  for (int j = threadIdx.x; j < 512; j += SWP * 64) {
    const int64_t c = (int64_t)blockIdx.x * 512 + j;
    if (c < C) {
      T t = red[0][j];
#pragma unroll
      for (int w = 1; w < SWP; ++w) t += red[w][j];
      dst[c] = t;
    }
  }
}

__global__ __launch_bounds__(AWP * 64) void k_absmean_partial_v8(const uint16_t* x, int64_t T, int64_t C, int64_t ld,
                                                                 int64_t tc, float* part) {
  __shared__ float red[AWP][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c0 = std::min<int64_t>((int64_t)blockIdx.x * 512 + lane * 8, C - 8);
  const int64_t t0 = (int64_t)blockIdx.y * tc, t1 = std::min<int64_t>(T, t0 + tc);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  stats_rows<AWP, QZ_ABSMEAN_NB>(x + c0, ld, t0, t1, wv, [&](const uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[2 * k] += fabsf(__uint_as_float(w[k] << 16));
      acc[2 * k + 1] += fabsf(__uint_as_float(w[k] & 0xffff0000u));
    }
  });
  stats_block_sum<AWP>(red, acc, lane, wv, C, part + (int64_t)blockIdx.y * C);
}
__global__ __launch_bounds__(256) void k_absmean_partial_v1(const uint16_t* x, int64_t T, int64_t C, int64_t ld,
                                                            int64_t tc, float* part) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const int64_t t0 = (int64_t)blockIdx.y * tc, t1 = std::min<int64_t>(T, t0 + tc);
  float acc = 0.f;
  for (int64_t t = t0; t < t1; ++t) acc += fabsf(bf2f(x[t * ld + c]));
  part[(int64_t)blockIdx.y * C + c] = acc;
}
// stage 2: block = 64 channels x FW waves; wave w sums chunks w, w+FW, ... (fixed order, loads
// unrolled so a lane has its chunks in flight together: the stage is latency-bound, ~nch*C*4 B),
// the FW wave sums are added in a fixed order; accumulated into sum[c]
constexpr int FW = 16;
template <typename T>
__global__ __launch_bounds__(FW * 64) void k_colsum_final(const T* part, int64_t nch, int64_t C, T* sum) {
  __shared__ T red[FW][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  T acc = 0;
  if (c < C) {
#pragma unroll 8
    for (int64_t k = wv; k < nch; k += FW) acc += part[k * C + c];
  }
  red[wv][lane] = acc;
  __syncthreads();
  if (wv == 0 && c < C) {
    T t = red[0][lane];
#pragma unroll
    for (int w = 1; w < FW; ++w) t += red[w][lane];
    sum[c] += t;
  }
}

// ---------------------------------------------- a3 / a4 in ONE launch (round 3)
// Column windows of WIN columns (lane = 8 columns, 16-B loads; a wave-load covers RPW =
// 64 / (WIN / 8) rows of WIN columns) x row chunks, as the two-launch kernels above, but the
// chunk partials are reduced INSIDE the launch by the last-arriving workgroups: chunks form
// groups of CPG; the last workgroup of a group to finish sums the group's partials (fixed
// order) into a group partial, and the last group to finish sums the group partials into
// sum[c].  No second kernel, no launch gap, and each reducing workgroup reads only CPG (or G)
// rows of the window.  Arrival counters live at the head of the caller's workspace (STATS_CNT
// words, zero before the first call; every last arriver resets its word, so every call leaves
// them zero).  Fixed order, hence deterministic: slot s = wave * RPW + (lane / (WIN / 8)) sums
// rows r0 + s, r0 + s + S, ... (S = SWP * RPW slots) in order; a chunk partial is
// ((slot 0 + slot 1) + ...) + slot S-1; a group partial and the final sum are each, over TF =
// NT / WIN thread groups f, ((sum_f=0 + sum_f=1) + ...) where sum_f adds items f, f + TF, ... of
// the group (chunks) / of the groups, in order.
constexpr int STATS_CNT = 8192;  // arrival counters (uint32) at the head of a statistics workspace
constexpr int64_t STATS_HEAD = (int64_t)STATS_CNT * 4;
static_assert(STATS_HEAD == QZ_STATS_HEAD_BYTES, "counter head of the statistics workspace (quantizers_amd.h)");
constexpr int QZ_STATS_CPG = 32; // chunks per first-level reduction group
constexpr int QZ_ABS1_WIN = 128; // absmean column window (128 / 256 / 512)
constexpr int QZ_ABS1_WPB = 8;
constexpr int QZ_ABS1_NB = 16; // rows per lane per walk batch ([16384, 4096]: a whole 512-token chunk in flight;
                        // 24.79 -> 24.35 us back to back, same bits: profiles/r04aj_tune_stats.log)
constexpr int QZ_ABS1_BLOCKS = 1024; // target workgroups of the one-launch absmean
constexpr int QZ_ABS1_MIN_RC = 256; // minimum tokens per chunk
constexpr int QZ_WM1_WIN = 128; // w_mean column window (at least the group size)
constexpr int QZ_WM1_WPB = 8;
constexpr int QZ_WM1_NB = 4;
constexpr int QZ_WM1_BLOCKS = 256; // target workgroups of the one-launch w_mean (power-of-two widths; wm1_blocks)
constexpr int QZ_WM1_MIN_RC = 128; // minimum rows per chunk

// rows rb + q, rb + q + S, ... < r1 of this lane's 8 columns (base = column pointer), SNB rows per
// batch, the next batch loaded before the current one is used; f(v, valid) per row in order.  rb
// is wave-uniform; every row of a batch that is followed by another batch is valid.  (Two
// register sets used in turn instead of the copy measured the same time with more VGPRs.)
constexpr int QZ_STATS_NT = 1; // non-temporal 16-B loads in the one-launch statistics walk: absmean 26.2 -> 25.0 us,
                        // w_mean 19.4 -> 18.1 us back to back, same bits (profiles/r04d_tune_stats.log)
template <int S, int SNB, typename F>
__device__ __forceinline__ void stats_walk(const uint16_t* base, int64_t ld, int64_t rb, int q, int64_t r1, F&& f) {
  if (rb >= r1) return;
  const uint32_t rlast = (uint32_t)(r1 - 1), uld = (uint32_t)ld;
  auto ld16 = [&](int64_t r) {
    const uint4* p = reinterpret_cast<const uint4*>(base + (uint64_t)std::min((uint32_t)r, rlast) * uld);
    if constexpr (QZ_STATS_NT) {
      return __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const qz_u32x4*>(p)));
    } else {
      return *p;
    }
  };
  constexpr int64_t STEP = (int64_t)SNB * S;
  uint4 a[SNB], b[SNB];
#pragma unroll
  for (int j = 0; j < SNB; ++j) a[j] = ld16(rb + q + (int64_t)j * S);
  for (; rb + STEP < r1; rb += STEP) {
#pragma unroll
    for (int j = 0; j < SNB; ++j) b[j] = ld16(rb + STEP + q + (int64_t)j * S);
#pragma unroll
    for (int j = 0; j < SNB; ++j) f(a[j], true);
#pragma unroll
    for (int j = 0; j < SNB; ++j) a[j] = b[j];
  }
#pragma unroll
  for (int j = 0; j < SNB; ++j) f(a[j], rb + q + (int64_t)j * S < r1);
}

// Memory ordering without a device-scope fence (an agent-scope release writes the whole L2 back
// and serialised a first version: 0.25-0.35 us per workgroup, profiles/r03b_tune_stats_fence.log):
// partials are written with agent-coherent (sc1) stores, every thread waits for its own stores
// to complete (s_waitcnt 0) before the workgroup barrier, thread 0 then arrives with a relaxed
// agent-scope atomic, and a last arriver reads the partials with agent-coherent loads.
template <typename T>
__device__ __forceinline__ void st_coherent(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// arrive at *c; true (on every thread) for the workgroup that completes `expect` arrivals
__device__ __forceinline__ bool arrive_last(unsigned* c, unsigned expect) {
  __shared__ int last;
  __builtin_amdgcn_s_waitcnt(0);  // this thread's coherent stores have completed
  __syncthreads();
  if (threadIdx.x == 0) last = __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == expect - 1;
  __syncthreads();
  const bool l = last;
  if (l && threadIdx.x == 0) __hip_atomic_store(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return l;
}
// fixed-order sum of rows src[i * C + c], i < n, for the window's columns: thread (j, f) adds
// rows f, f + TF, ... (coherent loads), then the TF sums are added in order; the result is valid
// in the threads with f == 0 (t = threadIdx.x)
template <int WIN, int NT, typename T>
__device__ __forceinline__ T reduce_rows(T (*red)[WIN], const T* src, int64_t n, int64_t C, int64_t cb) {
  constexpr int TF = NT / WIN;
  const int j = threadIdx.x % WIN, f = threadIdx.x / WIN;
  const int64_t c = cb + j;
  T t = 0;
  if (c < C) {
    // 8 coherent loads in flight, then added in order (the same order as one at a time)
    for (int64_t i0 = f; i0 < n; i0 += 8 * TF) {
      T v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int64_t i = i0 + (int64_t)k * TF;
        v[k] = i < n ? __hip_atomic_load(src + i * C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : T(0);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (i0 + (int64_t)k * TF < n) t += v[k];
    }
  }
  if constexpr (TF == 1) {
    return t;
  } else {
    __syncthreads();  // red may still be read by an earlier reduction
    red[f][j] = t;
    __syncthreads();
    T u = red[0][j];
#pragma unroll
    for (int k = 1; k < TF; ++k) u += red[k][j];
    return u;
  }
}

template <int WIN, int SWP, typename T>
__device__ __forceinline__ void stats_finish(T (*red)[WIN], const T* acc, int lane, int wv, int64_t C, int64_t nch,
                                             int64_t cpg, T* part, T* gpart, unsigned* cnt, T* sum, T pre, int64_t k) {
  constexpr int LPR = WIN / 8, RPW = 64 / LPR, S = SWP * RPW, NT = SWP * 64, TF = NT / WIN;
  static_assert(TF >= 1 && NT % WIN == 0 && S >= TF, "stats window");
  const int q = lane / LPR, c8 = lane % LPR;
#pragma unroll
  for (int i = 0; i < 8; ++i) red[wv * RPW + q][c8 * 8 + i] = acc[i];
  __syncthreads();
  const int64_t cb = (int64_t)blockIdx.x * WIN;
  for (int j = threadIdx.x; j < WIN; j += NT) {
    const int64_t c = cb + j;
    if (c < C) {
      T t = red[0][j];
#pragma unroll
      for (int s = 1; s < S; ++s) t += red[s][j];
      st_coherent(part + k * C + c, t);
    }
  }
  const int64_t ng = cdiv_d(nch, cpg), g = k / cpg, g0 = g * cpg;
  const int64_t n_g = std::min<int64_t>(cpg, nch - g0);
  unsigned* wc = cnt + blockIdx.x * (ng + 1);
  if (!arrive_last(wc + g, (unsigned)n_g)) return;
  const T vg = reduce_rows<WIN, NT>(red, part + g0 * C, n_g, C, cb);  // this group's chunks
  const bool out_thread = threadIdx.x < WIN && cb + threadIdx.x < C;
  if (ng == 1) {
    if (out_thread) sum[cb + threadIdx.x] = pre + vg;
    return;
  }
  if (out_thread) st_coherent(gpart + g * C + cb + threadIdx.x, vg);
  if (!arrive_last(wc + ng, (unsigned)ng)) return;
  const T v = reduce_rows<WIN, NT>(red, gpart, ng, C, cb);  // the groups, in order
  if (out_thread) sum[cb + threadIdx.x] = pre + v;
}

// the window's running sums, read when the workgroup starts: the last arriver's final add then
// waits for no load (only that workgroup writes them, after every workgroup of the window has
// started, so every copy is the value before this launch)
template <int WIN, typename T>
__device__ __forceinline__ T stats_pre(const T* sum, int64_t C) {
  const int64_t c = (int64_t)blockIdx.x * WIN + threadIdx.x;
  return (threadIdx.x < WIN && c < C) ? sum[c] : T(0);
}

// chunk k of one [T, C] operand (the whole launch, or one segment of a segmented launch)
template <int WIN>
__device__ __forceinline__ void absmean_chunk(float (*red)[WIN], const uint16_t* x, int64_t T, int64_t C, int64_t ld,
                                              int64_t tc, int64_t nch, int64_t cpg, float* part, float* gpart,
                                              unsigned* cnt, float* sum, int64_t k) {
  constexpr int SWP = QZ_ABS1_WPB, LPR = WIN / 8, RPW = 64 / LPR, S = SWP * RPW;
  // wave index through readfirstlane: known wave-uniform, so row bases stay in SGPRs
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane / LPR;
  const int64_t c0 = std::min<int64_t>((int64_t)blockIdx.x * WIN + (lane % LPR) * 8, C - 8);
  const int64_t t0 = k * tc, t1 = std::min<int64_t>(T, t0 + tc);
  const float pre = stats_pre<WIN>(sum, C);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto row = [&](const uint4 v, bool ok) {
    const uint32_t w[4] = {ok ? v.x : 0u, ok ? v.y : 0u, ok ? v.z : 0u, ok ? v.w : 0u};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[2 * k] += fabsf(__uint_as_float(w[k] << 16));
      acc[2 * k + 1] += fabsf(__uint_as_float(w[k] & 0xffff0000u));
    }
  };
  stats_walk<S, QZ_ABS1_NB>(x + c0, ld, t0 + wv * RPW, q, t1, row);
  stats_finish<WIN, SWP>(red, acc, lane, wv, C, nch, cpg, part, gpart, cnt, sum, pre, k);
}

template <int WIN>
__global__ __launch_bounds__(QZ_ABS1_WPB * 64) void k_absmean_1l(const uint16_t* x, int64_t T, int64_t C, int64_t ld,
                                                                int64_t tc, int64_t nch, int64_t cpg, float* part,
                                                                float* gpart, unsigned* cnt, float* sum) {
  __shared__ float red[QZ_ABS1_WPB * 64 / (WIN / 8)][WIN];
  absmean_chunk<WIN>(red, x, T, C, ld, tc, nch, cpg, part, gpart, cnt, sum, blockIdx.y);
}

// Segmented statistics (round 5): n independent operands of one column count in ONE launch --
// the calibration samples of one batched forward (absmean), the balance layers of one mapping
// (w_mean).  Segment s keeps exactly the chunking, workgroup order and reduction tree of its own
// single call (its chunks are grid rows chunk0[s] .. chunk0[s + 1] - 1, its partials, group
// partials and arrival counters their own slices of the workspace), so every out[s] is
// bit-identical to that call's result.
constexpr int QZ_STATS_SEGS = 16;
struct StatsSegs {
  const uint16_t* x[QZ_STATS_SEGS];
  void* out[QZ_STATS_SEGS];
  int64_t rows[QZ_STATS_SEGS], ld[QZ_STATS_SEGS], rc[QZ_STATS_SEGS], nch[QZ_STATS_SEGS];
  int64_t chunk0[QZ_STATS_SEGS + 1], gchunk0[QZ_STATS_SEGS], cnt0[QZ_STATS_SEGS];
  int32_t n;
};
__device__ __forceinline__ int seg_of(const StatsSegs& S, int64_t y) {  // wave-uniform
  int s = 0;
  while (s + 1 < S.n && y >= S.chunk0[s + 1]) ++s;
  return s;
}

template <int WIN>
__global__ __launch_bounds__(QZ_ABS1_WPB * 64) void k_absmean_seg(StatsSegs S, int64_t C, int64_t cpg, float* part,
                                                                 float* gpart, unsigned* cnt) {
  __shared__ float red[QZ_ABS1_WPB * 64 / (WIN / 8)][WIN];
  const int s = seg_of(S, blockIdx.y);
  absmean_chunk<WIN>(red, S.x[s], S.rows[s], C, S.ld[s], S.rc[s], S.nch[s], cpg, part + S.chunk0[s] * C,
                     gpart + S.gchunk0[s] * C, cnt + S.cnt0[s], (float*)S.out[s], blockIdx.y - S.chunk0[s]);
}

typedef float qz_f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 qz_bf16x2 __attribute__((ext_vector_type(2)));
// bf16(v) as an f32 in one convert: v_cvt_pk_bf16_f32(0, v) puts bf16(v) in the high half over
// a zero low half, which is the f32 value bf16(v) itself
__device__ __forceinline__ float bfr1(float v) {
  return __uint_as_float(__builtin_bit_cast(uint32_t, __builtin_convertvector((qz_f32x2){0.0f, v}, qz_bf16x2)));
}

template <int WIN, int LOGL>
__device__ __forceinline__ void wmean_chunk(double (*red)[WIN], const uint16_t* w, int64_t R, int64_t C, int64_t ld,
                                            int64_t rc, int64_t nch, int64_t cpg, double* part, double* gpart,
                                            unsigned* cnt, double* wsum, int64_t k) {
  constexpr int SWP = QZ_WM1_WPB, LPR = WIN / 8, RPW = 64 / LPR, S = SWP * RPW, L = 1 << LOGL;
  static_assert(L <= LPR, "a group must lie inside one row segment of the window");
  // wave index through readfirstlane: known wave-uniform, so row bases stay in SGPRs
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), q = lane / LPR;
  const int64_t c0 = std::min<int64_t>((int64_t)blockIdx.x * WIN + (lane % LPR) * 8, C - 8);
  const int64_t r0 = k * rc, r1 = std::min<int64_t>(R, r0 + rc);
  const double pre = stats_pre<WIN>(wsum, C);
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  auto row = [&](const uint4 v, bool ok) {
    const uint32_t u[4] = {v.x & 0x7fff7fffu, v.y & 0x7fff7fffu, v.z & 0x7fff7fffu, v.w & 0x7fff7fffu};
    // group absmax on |bf16| bit patterns (v_pk_max_u16 + DPP, every lane of the group on the same
    // row, so the group is uniformly valid or not), then |w| / bf16(amax + 1e-6)
    const uint32_t pm = pk_max_u16(pk_max_u16(u[0], u[1]), pk_max_u16(u[2], u[3]));
    const float m = __uint_as_float(grp_max_u<L>(max(pm & 0xffffu, pm >> 16)) << 16);
    const float rd = ok ? __builtin_amdgcn_rcpf(bfr1(m + 1e-6f)) : 0.f;  // rcp lemma; 0: adds +0.0
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[2 * k] += (double)bfr1(__uint_as_float(u[k] << 16) * rd);
      acc[2 * k + 1] += (double)bfr1(__uint_as_float(u[k] & 0xffff0000u) * rd);
    }
  };
  stats_walk<S, QZ_WM1_NB>(w + c0, ld, r0 + wv * RPW, q, r1, row);
  stats_finish<WIN, SWP>(red, acc, lane, wv, C, nch, cpg, part, gpart, cnt, wsum, pre, k);
}

template <int WIN, int LOGL>
__global__ __launch_bounds__(QZ_WM1_WPB * 64) void k_wmean_1l(const uint16_t* w, int64_t R, int64_t C, int64_t ld,
                                                             int64_t rc, int64_t nch, int64_t cpg, double* part,
                                                             double* gpart, unsigned* cnt, double* wsum) {
  __shared__ double red[QZ_WM1_WPB * 64 / (WIN / 8)][WIN];
  wmean_chunk<WIN, LOGL>(red, w, R, C, ld, rc, nch, cpg, part, gpart, cnt, wsum, blockIdx.y);
}

template <int WIN, int LOGL>
__global__ __launch_bounds__(QZ_WM1_WPB * 64) void k_wmean_seg(StatsSegs S, int64_t C, int64_t cpg, double* part,
                                                              double* gpart, unsigned* cnt) {
  __shared__ double red[QZ_WM1_WPB * 64 / (WIN / 8)][WIN];
  const int s = seg_of(S, blockIdx.y);
  wmean_chunk<WIN, LOGL>(red, S.x[s], S.rows[s], C, S.ld[s], S.rc[s], S.nch[s], cpg, part + S.chunk0[s] * C,
                         gpart + S.gchunk0[s] * C, cnt + S.cnt0[s], (double*)S.out[s], blockIdx.y - S.chunk0[s]);
}

// chunking of the one-launch kernels: >= min_rc rows per chunk, about `blocks` workgroups
int64_t stats1_chunks(int64_t R, int64_t C, int win, int64_t blocks, int64_t min_rc, int64_t* rc) {
  const int64_t bx = cdiv(C, win);
  const int64_t n = std::max<int64_t>(1, std::min<int64_t>(cdiv(R, min_rc), cdiv(blocks, bx)));
  *rc = cdiv(R, n);
  return cdiv(R, *rc);
}
int wmean_win(int64_t g) { return (int)std::min<int64_t>(512, std::max<int64_t>(QZ_WM1_WIN, g)); }
constexpr int ABS1_WIN = QZ_ABS1_WIN;
constexpr int ABS1_SWP = QZ_ABS1_WPB;
constexpr int WM1_SWP = QZ_WM1_WPB;
// workspace bytes of a one-launch statistics call: counters | chunk partials | group partials
int64_t stats1_bytes(int64_t nch, int64_t C, int64_t elem) {
  return STATS_HEAD + elem * (nch + cdiv(nch, QZ_STATS_CPG)) * C;
}
bool stats1_counters_fit(int64_t C, int win, int64_t nch) {
  return cdiv(C, win) * (cdiv(nch, QZ_STATS_CPG) + 1) <= STATS_CNT;
}

// ----------------------------------------------- a5: grid-search loss sum((a - b)^2)
// [3P] llmcompressor _compute_loss over a parent's outputs: (fp16_out - q_out) in the output
// dtype (bf16), squared in f32, summed (here in f64, fixed order: deterministic).
// stage 1: fixed grid, each thread walks 8-element units grid-stride, f64 partial per block
__device__ __forceinline__ double warp_sum_f64(double v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, WAVE);
  return v;
}
__global__ __launch_bounds__(256) void k_sqdiff_partial(const uint16_t* a, const uint16_t* b, int64_t rows,
                                                        int64_t cols, int64_t lda, int64_t ldb, int v8,
                                                        double* part) {
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  if (v8) {  // dense rows (lda == ldb == cols, cols % 8 == 0): flat 16-B units
    const int64_t n = rows * cols / 8;
    const uint4* A = reinterpret_cast<const uint4*>(a);
    const uint4* B = reinterpret_cast<const uint4*>(b);
    for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < n; u += stride) {
      const uint4 x = A[u], y = B[u];
      const uint32_t xa[4] = {x.x, x.y, x.z, x.w}, ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d0 = bfr(__uint_as_float(xa[k] << 16) - __uint_as_float(ya[k] << 16));
        const float d1 = bfr(__uint_as_float(xa[k] & 0xffff0000u) - __uint_as_float(ya[k] & 0xffff0000u));
        acc += (double)(d0 * d0);
        acc += (double)(d1 * d1);
      }
    }
  } else {
    const int64_t n = rows * cols;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += stride) {
      const int64_t r = e / cols, c = e - r * cols;
      const float d = bfr(bf2f(a[r * lda + c]) - bf2f(b[r * ldb + c]));
      acc += (double)(d * d);
    }
  }
  acc = warp_sum_f64(acc);
  __shared__ double red[256 / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) red[threadIdx.x / WAVE] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
// stage 2: one workgroup (4 waves) sums the partials in a fixed order (thread t: t, t+256, ...;
// then wave sums; then the 4 wave sums in order) and accumulates into *out
// blockIdx.x = loss i of a batched reduce: partial row part + i * part_ld -> out[i]
__global__ __launch_bounds__(256) void k_sqdiff_final(const double* part, int64_t nb, int64_t part_ld, double* out) {
  part += (int64_t)blockIdx.x * part_ld;
  out += blockIdx.x;
  double acc = 0.0;
#pragma unroll 4
  for (int64_t k = threadIdx.x; k < nb; k += 256) acc += part[k];
  acc = warp_sum_f64(acc);
  __shared__ double red[256 / WAVE];
  if ((threadIdx.x & (WAVE - 1)) == 0) red[threadIdx.x / WAVE] = acc;
  __syncthreads();
  if (threadIdx.x == 0) *out += ((red[0] + red[1]) + red[2]) + red[3];
}
// stage 1 for up to QZ_SQD_MULTI outputs b[0..G) against ONE shared reference a (dense rows):
// a unit of a is loaded once for all G outputs; output g is accumulated, reduced and stored
// exactly as k_sqdiff_partial's v8 path would for (a, b[g]) -> part[g * part_ld + block],
// so every loss keeps its bits while the reference is read once instead of G times
constexpr int QZ_SQD_MULTI = 8;
struct SqdOuts {
  const uint16_t* p[QZ_SQD_MULTI];
};
template <int G>
__global__ __launch_bounds__(256) void k_sqdiff_partial_multi(const uint16_t* a, SqdOuts B, int64_t n_units,
                                                              int64_t part_ld, double* part) {
  double acc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g] = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const uint4* A = reinterpret_cast<const uint4*>(a);
  for (int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x; u < n_units; u += stride) {
    const uint4 x = A[u];
    const uint32_t xa[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint4 y = reinterpret_cast<const uint4*>(B.p[g])[u];
      const uint32_t ya[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float d0 = bfr(__uint_as_float(xa[k] << 16) - __uint_as_float(ya[k] << 16));
        const float d1 = bfr(__uint_as_float(xa[k] & 0xffff0000u) - __uint_as_float(ya[k] & 0xffff0000u));
        acc[g] += (double)(d0 * d0);
        acc[g] += (double)(d1 * d1);
      }
    }
  }
  __shared__ double red[G][256 / WAVE];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const double v = warp_sum_f64(acc[g]);
    if ((threadIdx.x & (WAVE - 1)) == 0) red[g][threadIdx.x / WAVE] = v;
  }
  __syncthreads();
  if (threadIdx.x < G) {
    const int g = threadIdx.x;
    part[(int64_t)g * part_ld + blockIdx.x] = red[g][0] + red[g][1] + red[g][2] + red[g][3];
  }
}
template <int G>
void launch_sqd_multi(const uint16_t* a, const SqdOuts& B, int64_t n_units, int64_t nb, int64_t part_ld, double* part,
                      hipStream_t st) {
  hipLaunchKernelGGL(k_sqdiff_partial_multi<G>, dim3((unsigned)nb), dim3(256), 0, st, a, B, n_units, part_ld, part);
}
int64_t sqdiff_blocks(int64_t rows, int64_t cols) {
  return std::max<int64_t>(1, std::min<int64_t>(2048, cdiv(rows * cols, 256 * 8 * 4)));
}

constexpr int QZ_ABSMEAN_MIN_TC = 128; // minimum tokens per stage-1 chunk
constexpr int QZ_ABSMEAN_BLOCKS = 1024; // target stage-1 workgroups
int64_t absmean_chunks(int64_t T, int64_t C, int64_t* tc) {
  // >= QZ_ABSMEAN_MIN_TC tokens per chunk (32 per wave: one round of 8 loads); about
  // QZ_ABSMEAN_BLOCKS stage-1 blocks
  const int64_t bx = cdiv(C, 512);
  int64_t nch = std::max<int64_t>(1, std::min<int64_t>(cdiv(T, QZ_ABSMEAN_MIN_TC), cdiv(QZ_ABSMEAN_BLOCKS, bx)));
  *tc = cdiv(T, nch);
  return cdiv(T, *tc);
}

constexpr int QZ_WMEAN_BLOCKS = 256; // target stage-1 workgroups of w_mean
constexpr int QZ_WMEAN_MIN_RC = 16; // minimum rows per stage-1 chunk
// row chunks of the w_mean stage 1: >= QZ_WMEAN_MIN_RC rows each, about QZ_WMEAN_BLOCKS workgroups
int64_t wmean_chunks(int64_t R, int64_t C, int64_t* rc) {
  const int64_t bx = cdiv(C, 512);
  const int64_t nrc = std::max<int64_t>(1, std::min<int64_t>(cdiv(R, QZ_WMEAN_MIN_RC), cdiv(QZ_WMEAN_BLOCKS, bx)));
  *rc = cdiv(R, nrc);
  return cdiv(R, *rc);
}

// ------------------------------------------------- a4: w_mean numerator (f64 sums)
// stage 1: the stats_rows walk above over the weight rows (a group of L = g/8 lanes is inside one
// 512-column window, so lanes whose columns were clamped form whole groups and only compute
// discarded sums); per row the group absmax by DPP, then |w| / bf16(absmax + 1e-6) in bf16,
// summed in f64 -> part[row chunk][c].  Stage 2 (k_colsum_final) adds the chunks in order.
template <int LOGL>
__global__ __launch_bounds__(WWP * 64) void k_wmean_v8(const uint16_t* w, int64_t R, int64_t C, int64_t ld, int64_t rc,
                                                       double* part) {
  constexpr int L = 1 << LOGL;
  __shared__ double red[WWP][512];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t c0 = std::min<int64_t>((int64_t)blockIdx.x * 512 + lane * 8, C - 8);
  const int64_t r0 = (int64_t)blockIdx.y * rc, r1 = std::min<int64_t>(R, r0 + rc);
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  stats_rows<WWP, QZ_WMEAN_NB>(w + c0, ld, r0, r1, wv, [&](const uint4 v) {
    const uint32_t u[4] = {v.x & 0x7fff7fffu, v.y & 0x7fff7fffu, v.z & 0x7fff7fffu, v.w & 0x7fff7fffu};
    // group absmax on |bf16| bit patterns (v_pk_max_u16 + DPP), then |w| / bf16(amax + 1e-6)
    const uint32_t pm = pk_max_u16(pk_max_u16(u[0], u[1]), pk_max_u16(u[2], u[3]));
    const float m = __uint_as_float(grp_max_u<L>(max(pm & 0xffffu, pm >> 16)) << 16);
    const float d = bfr(m + 1e-6f);
    const float rd = __builtin_amdgcn_rcpf(d);  // bf16(|w| * rcp(d)) == bf16(|w| / d): rcp lemma
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc[2 * k] += (double)bfr(__uint_as_float(u[k] << 16) * rd);
      acc[2 * k + 1] += (double)bfr(__uint_as_float(u[k] & 0xffff0000u) * rd);
    }
  });
  stats_block_sum<WWP>(red, acc, lane, wv, C, part + (int64_t)blockIdx.y * C);
}
// generic: one thread per column walks every row in order (deterministic); any group size /
// alignment
__global__ void k_wmean_generic(const uint16_t* w, int64_t R, int64_t C, int64_t ld, int64_t g, double* wsum) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const int64_t gc0 = (c / g) * g;
  double acc = 0.0;
  for (int64_t r = 0; r < R; ++r) {
    float m = 0.f;
    for (int64_t k = 0; k < g; ++k) m = fmaxf(m, fabsf(bf2f(w[r * ld + gc0 + k])));
    const float d = bfr(m + 1e-6f);
    acc += (double)bfr(fabsf(bf2f(w[r * ld + c])) / d);
  }
  wsum[c] += acc;
}

// ------------------------------------------------------- a5: one grid point's scales
__device__ __forceinline__ float nmax(float a, float b) { return (a != a || b != b) ? NAN : fmaxf(a, b); }
__device__ __forceinline__ float nmin(float a, float b) { return (a != a || b != b) ? NAN : fminf(a, b); }

__global__ __launch_bounds__(1024) void k_grid_scales(const float* xm, const float* wm, int64_t C, float ratio,
                                                      int duo, float* out) {
  // one workgroup per scale vector (blockIdx.x = batch item: one MoE expert's mapping)
  xm += (int64_t)blockIdx.x * C;
  if (wm) wm += (int64_t)blockIdx.x * C;
  out += (int64_t)blockIdx.x * C;
  __shared__ float smx[16], smn[16];
  float lmx = -INFINITY, lmn = INFINITY;
  for (int64_t c = threadIdx.x; c < C; c += 1024) {
    float s = powf(xm[c], ratio);
    if (duo) s = s / (powf(wm[c], 1.0f - ratio) + 1e-4f);
    s = (s != s) ? s : fmaxf(s, 1e-4f);  // clamp(min=1e-4), NaN propagates
    out[c] = s;
    lmx = nmax(lmx, s);
    lmn = nmin(lmn, s);
  }
  for (int m = 1; m < 64; m <<= 1) {
    lmx = nmax(lmx, __shfl_xor(lmx, m, WAVE));
    lmn = nmin(lmn, __shfl_xor(lmn, m, WAVE));
  }
  if ((threadIdx.x & 63) == 0) { smx[threadIdx.x >> 6] = lmx; smn[threadIdx.x >> 6] = lmn; }
  __syncthreads();
  float gmx = smx[0], gmn = smn[0];
  for (int k = 1; k < 16; ++k) { gmx = nmax(gmx, smx[k]); gmn = nmin(gmn, smn[k]); }
  const float norm = sqrtf(gmx * gmn);
  for (int64_t c = threadIdx.x; c < C; c += 1024) {
    float s = out[c] / norm;
    if (s != s || fabsf(s) == INFINITY) s = 1.0f;
    out[c] = s;
  }
}

// --------------------------------------------------------------- a6: smoothing
__global__ void k_scale_cols(uint16_t* w, int64_t R, int64_t C, int64_t ld, const float* s, int divide) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= R * C) return;
  const int64_t r = e / C, c = e % C;
  uint16_t* p = w + r * ld + c;
  const float x = bf2f(*p);
  *p = f2bf(divide ? x / s[c] : x * s[c]);
}
__global__ void k_scale_rows(uint16_t* w, int64_t R, int64_t C, int64_t ld, const float* s, int divide) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= R * C) return;
  const int64_t r = e / C, c = e % C;
  uint16_t* p = w + r * ld + c;
  const float x = bf2f(*p);
  *p = f2bf(divide ? x / s[r] : x * s[r]);
}

// 8 bf16 per thread (one 16-B access), grid (column octets, rows); column scales as 2 float4
template <bool COLS>
__global__ __launch_bounds__(256) void k_scale_v8(uint16_t* w, int64_t R, int64_t C, int64_t ld, const float* s,
                                                  int divide) {
  const int64_t c8 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c8 * 8 >= C) return;
  float cs[8];
  if (COLS) {
    const float4 a = *reinterpret_cast<const float4*>(s + c8 * 8);
    const float4 b = *reinterpret_cast<const float4*>(s + c8 * 8 + 4);
    cs[0] = a.x; cs[1] = a.y; cs[2] = a.z; cs[3] = a.w; cs[4] = b.x; cs[5] = b.y; cs[6] = b.z; cs[7] = b.w;
  }
  for (int64_t r = blockIdx.y; r < R; r += gridDim.y) {
    uint4* p = reinterpret_cast<uint4*>(w + r * ld + c8 * 8);
    const uint4 v = *p;
    const uint32_t u[4] = {v.x, v.y, v.z, v.w};
    uint32_t o[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x0 = __uint_as_float(u[k] << 16), x1 = __uint_as_float(u[k] & 0xffff0000u);
      const float s0 = COLS ? cs[2 * k] : s[r], s1 = COLS ? cs[2 * k + 1] : s[r];
      const float y0 = divide ? x0 / s0 : x0 * s0, y1 = divide ? x1 / s1 : x1 * s1;
      o[k] = (uint32_t)f2bf(y0) | ((uint32_t)f2bf(y1) << 16);
    }
    st16_wt(p, make_uint4(o[0], o[1], o[2], o[3]));
  }
}

bool v8_ok(const void* w, int64_t C, int64_t ld, const float* s, bool cols) {
  return C % 8 == 0 && ld % 8 == 0 && aligned(w, 16) && (!cols || aligned(s, 16));
}

}  // namespace

extern "C" {

// one-launch plan of an absmean call (chunks), or -1 when the counters do not fit (two-launch path)
static int64_t absmean_1l(int64_t tokens, int64_t channels, int64_t* tc) {
  const int64_t n1 = stats1_chunks(tokens, channels, ABS1_WIN, QZ_ABS1_BLOCKS, QZ_ABS1_MIN_RC, tc);
  return stats1_counters_fit(channels, ABS1_WIN, n1) ? n1 : -1;
}

size_t qz_awq_absmean_workspace_size(int64_t tokens, int64_t channels) {
  if (tokens <= 0 || channels <= 0) return 0;
  int64_t tc, tc1;
  const int64_t nch = absmean_chunks(tokens, channels, &tc);  // the two-launch path's slab
  const int64_t n1 = absmean_1l(tokens, channels, &tc1);
  if (n1 > 0)  // (the two-launch path still serves unaligned inputs, after the counters)
    return (size_t)std::max<int64_t>(stats1_bytes(n1, channels, 4), STATS_HEAD + 4 * nch * channels);
  return (size_t)4 * (size_t)(nch * channels);
}

int qz_awq_absmean_accum(const void* x, int64_t tokens, int64_t channels, int64_t ld, float* sum, void* workspace,
                         size_t workspace_bytes, qz_stream_t stream) {
  if (!x || !sum) return QZ_ERR_NULL;
  if (tokens < 0 || channels <= 0 || ld < channels) return QZ_ERR_SHAPE;
  if (tokens == 0) return QZ_OK;
  if (!workspace || workspace_bytes < qz_awq_absmean_workspace_size(tokens, channels)) return QZ_ERR_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  int64_t tc, tc1;
  const int64_t nch = absmean_chunks(tokens, channels, &tc);
  const int64_t n1 = absmean_1l(tokens, channels, &tc1);
  float* part = (float*)workspace;
  const bool v8 = channels % 8 == 0 && ld % 8 == 0 && aligned(x, 16) && aligned(workspace, 16) &&
                  tokens < INT32_MAX && ld < INT32_MAX;
  if (v8 && n1 > 0) {
    float* p1 = (float*)((char*)workspace + STATS_HEAD);
    hipLaunchKernelGGL(k_absmean_1l<ABS1_WIN>, dim3((unsigned)cdiv(channels, ABS1_WIN), (unsigned)n1),
                       dim3(QZ_ABS1_WPB * 64), 0, st, (const uint16_t*)x, tokens, channels, ld, tc1, n1,
                       (int64_t)QZ_STATS_CPG, p1, p1 + n1 * channels, (unsigned*)workspace, sum);
    return launch_err();
  }
  if (n1 > 0) part = (float*)((char*)workspace + STATS_HEAD);  // same workspace layout
  if (v8) {
    dim3 grid((unsigned)cdiv(channels, 512), (unsigned)nch);
    hipLaunchKernelGGL(k_absmean_partial_v8, grid, dim3(AWP * 64), 0, st, (const uint16_t*)x, tokens, channels, ld, tc, part);
  } else {
    dim3 grid((unsigned)cdiv(channels, 256), (unsigned)nch);
    hipLaunchKernelGGL(k_absmean_partial_v1, grid, dim3(256), 0, st, (const uint16_t*)x, tokens, channels, ld, tc, part);
  }
  int rc = launch_err();
  if (rc) return rc;
  hipLaunchKernelGGL(k_colsum_final<float>, dim3((unsigned)cdiv(channels, 64)), dim3(FW * 64), 0, st, part, nch, channels,
                     sum);
  return launch_err();
}

size_t qz_awq_sq_err_workspace_size(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return (size_t)8 * (size_t)sqdiff_blocks(rows, cols);
}

int qz_awq_sq_err_accum(const void* a, const void* b, int64_t rows, int64_t cols, int64_t lda, int64_t ldb,
                        double* out, void* workspace, size_t workspace_bytes, qz_stream_t stream) {
  if (!a || !b || !out) return QZ_ERR_NULL;
  if (rows < 0 || cols <= 0 || lda < cols || ldb < cols) return QZ_ERR_SHAPE;
  if (rows == 0) return QZ_OK;
  if (!workspace || workspace_bytes < qz_awq_sq_err_workspace_size(rows, cols)) return QZ_ERR_WORKSPACE;
  const int64_t nb = sqdiff_blocks(rows, cols);
  const int v8 = lda == cols && ldb == cols && cols % 8 == 0 && aligned(a, 16) && aligned(b, 16);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_sqdiff_partial, dim3((unsigned)nb), dim3(256), 0, st, (const uint16_t*)a, (const uint16_t*)b,
                     rows, cols, lda, ldb, v8, (double*)workspace);
  int rc = launch_err();
  if (rc) return rc;
  hipLaunchKernelGGL(k_sqdiff_final, dim3(1), dim3(256), 0, st, (const double*)workspace, nb, (int64_t)0, out);
  return launch_err();
}

int64_t qz_awq_sq_err_partials_count(int64_t rows, int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  return sqdiff_blocks(rows, cols);
}

int qz_awq_sq_err_partials(const void* a, const void* b, int64_t rows, int64_t cols, int64_t lda, int64_t ldb,
                           double* part, qz_stream_t stream) {
  if (!a || !b || !part) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0 || lda < cols || ldb < cols) return QZ_ERR_SHAPE;
  if (!aligned(part, 8)) return QZ_ERR_ALIGN;
  const int64_t nb = sqdiff_blocks(rows, cols);
  const int v8 = lda == cols && ldb == cols && cols % 8 == 0 && aligned(a, 16) && aligned(b, 16);
  hipLaunchKernelGGL(k_sqdiff_partial, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, (const uint16_t*)a,
                     (const uint16_t*)b, rows, cols, lda, ldb, v8, part);
  return launch_err();
}

int qz_awq_sq_err_partials_multi(const void* a, const void* const* b, int32_t n_b, int64_t rows, int64_t cols,
                                 double* part, int64_t part_ld, qz_stream_t stream) {
  if (!a || !b || !part) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0 || cols % 8 || n_b < 1 || n_b > QZ_SQD_MULTI) return QZ_ERR_SHAPE;
  const int64_t nb = sqdiff_blocks(rows, cols);
  if (part_ld < nb) return QZ_ERR_SHAPE;
  if (!aligned(part, 8) || !aligned(a, 16)) return QZ_ERR_ALIGN;
  SqdOuts B = {};
  for (int g = 0; g < n_b; ++g) {
    if (!b[g]) return QZ_ERR_NULL;
    if (!aligned(b[g], 16)) return QZ_ERR_ALIGN;
    B.p[g] = (const uint16_t*)b[g];
  }
  const uint16_t* ap = (const uint16_t*)a;
  const int64_t n = rows * cols / 8;
  hipStream_t st = (hipStream_t)stream;
  switch (n_b) {
    case 1: launch_sqd_multi<1>(ap, B, n, nb, part_ld, part, st); break;
    case 2: launch_sqd_multi<2>(ap, B, n, nb, part_ld, part, st); break;
    case 3: launch_sqd_multi<3>(ap, B, n, nb, part_ld, part, st); break;
    case 4: launch_sqd_multi<4>(ap, B, n, nb, part_ld, part, st); break;
    case 5: launch_sqd_multi<5>(ap, B, n, nb, part_ld, part, st); break;
    case 6: launch_sqd_multi<6>(ap, B, n, nb, part_ld, part, st); break;
    case 7: launch_sqd_multi<7>(ap, B, n, nb, part_ld, part, st); break;
    default: launch_sqd_multi<8>(ap, B, n, nb, part_ld, part, st); break;
  }
  return launch_err();
}

int qz_awq_sq_err_reduce(const double* part, int64_t n, int64_t nb, int64_t part_ld, double* out, qz_stream_t stream) {
  if (n == 0) return QZ_OK;
  if (!part || !out) return QZ_ERR_NULL;
  if (n < 0 || nb <= 0 || part_ld < nb || n > INT32_MAX) return QZ_ERR_SHAPE;
  if (!aligned(part, 8) || !aligned(out, 8)) return QZ_ERR_ALIGN;
  hipLaunchKernelGGL(k_sqdiff_final, dim3((unsigned)n), dim3(256), 0, (hipStream_t)stream, part, nb, part_ld, out);
  return launch_err();
}

// target workgroups of a one-launch w_mean: 256 when the row pitch is a power of two, else 512
// (1024 from 96 MB).  profiles/r05i-k_tune_stats*: at 256 workgroups rows of 2560 / 3072 columns
// stream at 3.3-3.9 TB/s against 5-5.8 TB/s for 2048 / 4096; more row chunks recover most of it
// ([19456, 2560]: 29.8 -> 23.9 us; [9728, 2560]: 17.1 -> 15.2 us; [24576, 3072]: 41.4 -> 34.4
// us) while power-of-two widths lose with them ([11008, 4096]: 18.0 -> 20.4 us)
static int64_t wm1_blocks(int64_t rows, int64_t cols) {
  if ((cols & (cols - 1)) == 0) return QZ_WM1_BLOCKS;
  return rows * cols * 2 >= (96ll << 20) ? 4 * QZ_WM1_BLOCKS : 2 * QZ_WM1_BLOCKS;
}
// one-launch plan of a w_mean call (chunks), or -1 (two-launch / generic paths)
static int64_t wmean_1l(int64_t rows, int64_t cols, int64_t g, int64_t* rc) {
  if (g < 8 || g > 512 || (g & (g - 1))) return -1;
  const int win = wmean_win(g);
  const int64_t n1 = stats1_chunks(rows, cols, win, wm1_blocks(rows, cols), QZ_WM1_MIN_RC, rc);
  return stats1_counters_fit(cols, win, n1) ? n1 : -1;
}

size_t qz_awq_weight_mean_workspace_size(int64_t rows, int64_t cols, int32_t group_size) {
  if (rows <= 0 || cols <= 0 || group_size <= 0) return 0;
  int64_t rc;
  const int64_t n1 = wmean_1l(rows, cols, group_size, &rc);
  if (n1 > 0) return (size_t)stats1_bytes(n1, cols, 8);
  return (size_t)8 * (size_t)(wmean_chunks(rows, cols, &rc) * cols);
}

extern "C++" {
template <int WIN>
static void launch_wmean_1l(int logl, dim3 grid, dim3 blk, hipStream_t st, const uint16_t* wp, int64_t rows, int64_t cols,
                            int64_t ld, int64_t rc, int64_t n1, double* p1, unsigned* cnt, double* wsum) {
  double* gp = p1 + n1 * cols;
  const int64_t cpg = QZ_STATS_CPG;
  switch (logl) {
    case 0: hipLaunchKernelGGL((k_wmean_1l<WIN, 0>), grid, blk, 0, st, wp, rows, cols, ld, rc, n1, cpg, p1, gp, cnt, wsum); break;
    case 1: hipLaunchKernelGGL((k_wmean_1l<WIN, 1>), grid, blk, 0, st, wp, rows, cols, ld, rc, n1, cpg, p1, gp, cnt, wsum); break;
    case 2: hipLaunchKernelGGL((k_wmean_1l<WIN, 2>), grid, blk, 0, st, wp, rows, cols, ld, rc, n1, cpg, p1, gp, cnt, wsum); break;
    case 3: hipLaunchKernelGGL((k_wmean_1l<WIN, 3>), grid, blk, 0, st, wp, rows, cols, ld, rc, n1, cpg, p1, gp, cnt, wsum); break;
    case 4: hipLaunchKernelGGL((k_wmean_1l<WIN, 4>), grid, blk, 0, st, wp, rows, cols, ld, rc, n1, cpg, p1, gp, cnt, wsum); break;
    case 5:
      if constexpr (WIN >= 256)
        hipLaunchKernelGGL((k_wmean_1l<WIN, 5>), grid, blk, 0, st, wp, rows, cols, ld, rc, n1, cpg, p1, gp, cnt, wsum);
      break;
    default:
      if constexpr (WIN >= 512)
        hipLaunchKernelGGL((k_wmean_1l<WIN, 6>), grid, blk, 0, st, wp, rows, cols, ld, rc, n1, cpg, p1, gp, cnt, wsum);
      break;
  }
}
}  // extern "C++"

int qz_awq_weight_mean_accum(const void* w, int64_t rows, int64_t cols, int64_t ld, int32_t group_size, double* wsum,
                             void* workspace, size_t workspace_bytes, qz_stream_t stream) {
  if (!w || !wsum) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0 || ld < cols) return QZ_ERR_SHAPE;
  if (group_size <= 0 || cols % group_size) return QZ_ERR_GROUP;
  hipStream_t st = (hipStream_t)stream;
  const int64_t g = group_size;
  const bool pow2 = g >= 8 && g <= 512 && (g & (g - 1)) == 0;
  if (pow2 && ld % 8 == 0 && aligned(w, 16) && rows < INT32_MAX && ld < INT32_MAX) {
    if (!workspace || workspace_bytes < qz_awq_weight_mean_workspace_size(rows, cols, group_size))
      return QZ_ERR_WORKSPACE;
    if (!aligned(workspace, 8)) return QZ_ERR_ALIGN;
    int logl = 0;
    while ((8 << logl) < g) ++logl;
    const uint16_t* wp = (const uint16_t*)w;
    int64_t rc1;
    const int64_t n1 = wmean_1l(rows, cols, g, &rc1);
    if (n1 > 0) {
      const int win = wmean_win(g);
      dim3 grid1((unsigned)cdiv(cols, win), (unsigned)n1), blk1(QZ_WM1_WPB * 64);
      double* p1 = (double*)((char*)workspace + STATS_HEAD);
      unsigned* cnt = (unsigned*)workspace;
      if (win == 512) launch_wmean_1l<512>(logl, grid1, blk1, st, wp, rows, cols, ld, rc1, n1, p1, cnt, wsum);
      else if (win == 256) launch_wmean_1l<256>(logl, grid1, blk1, st, wp, rows, cols, ld, rc1, n1, p1, cnt, wsum);
      else launch_wmean_1l<128>(logl, grid1, blk1, st, wp, rows, cols, ld, rc1, n1, p1, cnt, wsum);
      return launch_err();
    }
    int64_t rc;
    const int64_t nch = wmean_chunks(rows, cols, &rc);
    dim3 grid((unsigned)cdiv(cols, 512), (unsigned)nch);
    double* part = (double*)workspace;
    switch (logl) {
      case 0: hipLaunchKernelGGL(k_wmean_v8<0>, grid, dim3(WWP * 64), 0, st, wp, rows, cols, ld, rc, part); break;
      case 1: hipLaunchKernelGGL(k_wmean_v8<1>, grid, dim3(WWP * 64), 0, st, wp, rows, cols, ld, rc, part); break;
      case 2: hipLaunchKernelGGL(k_wmean_v8<2>, grid, dim3(WWP * 64), 0, st, wp, rows, cols, ld, rc, part); break;
      case 3: hipLaunchKernelGGL(k_wmean_v8<3>, grid, dim3(WWP * 64), 0, st, wp, rows, cols, ld, rc, part); break;
      case 4: hipLaunchKernelGGL(k_wmean_v8<4>, grid, dim3(WWP * 64), 0, st, wp, rows, cols, ld, rc, part); break;
      case 5: hipLaunchKernelGGL(k_wmean_v8<5>, grid, dim3(WWP * 64), 0, st, wp, rows, cols, ld, rc, part); break;
      default: hipLaunchKernelGGL(k_wmean_v8<6>, grid, dim3(WWP * 64), 0, st, wp, rows, cols, ld, rc, part); break;
    }
    int e = launch_err();
    if (e) return e;
    hipLaunchKernelGGL(k_colsum_final<double>, dim3((unsigned)cdiv(cols, 64)), dim3(FW * 64), 0, st, part, nch, cols,
                       wsum);
  } else {
    hipLaunchKernelGGL(k_wmean_generic, dim3((unsigned)cdiv(cols, 256)), dim3(256), 0, st, (const uint16_t*)w, rows,
                       cols, ld, g, wsum);
  }
  return launch_err();
}

// the segment table of a segmented call: every segment on its single call's one-launch plan;
// false when one is not (the caller then issues single calls)
static bool segs_plan(int which, int32_t n, const int64_t* rows, int64_t cols, int32_t g, StatsSegs* S,
                      int64_t* ws_bytes) {
  if (n < 1 || n > QZ_STATS_SEGS || cols <= 0 || !rows) return false;
  const int win = which == 0 ? ABS1_WIN : wmean_win(g);
  const int64_t bx = cdiv(cols, win), elem = which == 0 ? 4 : 8;
  int64_t chunks = 0, groups = 0, cnts = 0;
  S->n = n;
  for (int s = 0; s < n; ++s) {
    if (rows[s] <= 0 || rows[s] >= INT32_MAX) return false;
    int64_t rc = 0;
    const int64_t n1 = which == 0 ? absmean_1l(rows[s], cols, &rc) : wmean_1l(rows[s], cols, g, &rc);
    if (n1 <= 0) return false;
    const int64_t ng = cdiv(n1, QZ_STATS_CPG);
    S->rows[s] = rows[s];
    S->rc[s] = rc;
    S->nch[s] = n1;
    S->chunk0[s] = chunks;
    S->gchunk0[s] = groups;
    S->cnt0[s] = cnts;
    chunks += n1;
    groups += ng;
    cnts += bx * (ng + 1);
  }
  S->chunk0[n] = chunks;
  if (cnts > STATS_CNT || chunks > 65535) return false;
  *ws_bytes = STATS_HEAD + elem * (chunks + groups) * cols;
  return true;
}

static bool segs_inputs_ok(int32_t n, const void* const* x, const int64_t* ld, int64_t cols, void* const* out,
                           size_t out_align) {
  if (cols % 8) return false;
  for (int s = 0; s < n; ++s) {
    if (!x[s] || !out[s] || !aligned(x[s], 16) || !aligned(out[s], out_align) || ld[s] < cols || ld[s] % 8 ||
        ld[s] >= INT32_MAX)
      return false;
    for (int t = 0; t < s; ++t)
      if (out[t] == out[s]) return false;  // each segment its own sums (no two reducers on one row)
  }
  return true;
}

size_t qz_awq_absmean_segments_workspace_size(int32_t n, const int64_t* tokens, int64_t channels) {
  StatsSegs S;
  int64_t b = 0;
  return segs_plan(0, n, tokens, channels, 0, &S, &b) ? (size_t)b : 0;
}

int qz_awq_absmean_accum_segments(int32_t n, const void* const* x, const int64_t* tokens, int64_t channels,
                                  const int64_t* ld, float* const* sums, void* workspace, size_t workspace_bytes,
                                  qz_stream_t stream) {
  if (!x || !tokens || !ld || !sums) return QZ_ERR_NULL;
  StatsSegs S;
  int64_t need = 0;
  if (!segs_plan(0, n, tokens, channels, 0, &S, &need) ||
      !segs_inputs_ok(n, x, ld, channels, (void* const*)sums, 4))
    return QZ_ERR_FORMAT;
  if (!workspace || (int64_t)workspace_bytes < need) return QZ_ERR_WORKSPACE;
  if (!aligned(workspace, 16)) return QZ_ERR_ALIGN;
  for (int s = 0; s < n; ++s) {
    S.x[s] = (const uint16_t*)x[s];
    S.ld[s] = ld[s];
    S.out[s] = sums[s];
  }
  float* p1 = (float*)((char*)workspace + STATS_HEAD);
  hipLaunchKernelGGL(k_absmean_seg<ABS1_WIN>, dim3((unsigned)cdiv(channels, ABS1_WIN), (unsigned)S.chunk0[n]),
                     dim3(QZ_ABS1_WPB * 64), 0, (hipStream_t)stream, S, channels, (int64_t)QZ_STATS_CPG, p1,
                     p1 + S.chunk0[n] * channels, (unsigned*)workspace);
  return launch_err();
}

size_t qz_awq_weight_mean_segments_workspace_size(int32_t n, const int64_t* rows, int64_t cols, int32_t group_size) {
  StatsSegs S;
  int64_t b = 0;
  return segs_plan(1, n, rows, cols, group_size, &S, &b) ? (size_t)b : 0;
}

extern "C++" {
template <int WIN>
static void launch_wmean_seg(int logl, dim3 grid, dim3 blk, hipStream_t st, const StatsSegs& S, int64_t cols,
                             double* p1, double* gp, unsigned* cnt) {
  const int64_t cpg = QZ_STATS_CPG;
  switch (logl) {
    case 0: hipLaunchKernelGGL((k_wmean_seg<WIN, 0>), grid, blk, 0, st, S, cols, cpg, p1, gp, cnt); break;
    case 1: hipLaunchKernelGGL((k_wmean_seg<WIN, 1>), grid, blk, 0, st, S, cols, cpg, p1, gp, cnt); break;
    case 2: hipLaunchKernelGGL((k_wmean_seg<WIN, 2>), grid, blk, 0, st, S, cols, cpg, p1, gp, cnt); break;
    case 3: hipLaunchKernelGGL((k_wmean_seg<WIN, 3>), grid, blk, 0, st, S, cols, cpg, p1, gp, cnt); break;
    case 4: hipLaunchKernelGGL((k_wmean_seg<WIN, 4>), grid, blk, 0, st, S, cols, cpg, p1, gp, cnt); break;
    case 5:
      if constexpr (WIN >= 256) hipLaunchKernelGGL((k_wmean_seg<WIN, 5>), grid, blk, 0, st, S, cols, cpg, p1, gp, cnt);
      break;
    default:
      if constexpr (WIN >= 512) hipLaunchKernelGGL((k_wmean_seg<WIN, 6>), grid, blk, 0, st, S, cols, cpg, p1, gp, cnt);
      break;
  }
}
}  // extern "C++"

int qz_awq_weight_mean_accum_segments(int32_t n, const void* const* w, const int64_t* rows, int64_t cols,
                                      const int64_t* ld, int32_t group_size, double* const* wsums, void* workspace,
                                      size_t workspace_bytes, qz_stream_t stream) {
  if (!w || !rows || !ld || !wsums) return QZ_ERR_NULL;
  if (group_size <= 0 || cols % group_size) return QZ_ERR_GROUP;
  StatsSegs S;
  int64_t need = 0;
  if (!segs_plan(1, n, rows, cols, group_size, &S, &need) ||
      !segs_inputs_ok(n, w, ld, cols, (void* const*)wsums, 8))
    return QZ_ERR_FORMAT;
  if (!workspace || (int64_t)workspace_bytes < need) return QZ_ERR_WORKSPACE;
  if (!aligned(workspace, 8)) return QZ_ERR_ALIGN;
  for (int s = 0; s < n; ++s) {
    S.x[s] = (const uint16_t*)w[s];
    S.ld[s] = ld[s];
    S.out[s] = wsums[s];
  }
  int logl = 0;
  while ((8 << logl) < group_size) ++logl;
  const int win = wmean_win(group_size);
  const dim3 grid((unsigned)cdiv(cols, win), (unsigned)S.chunk0[n]), blk(QZ_WM1_WPB * 64);
  double* p1 = (double*)((char*)workspace + STATS_HEAD);
  double* gp = p1 + S.chunk0[n] * cols;
  hipStream_t st = (hipStream_t)stream;
  if (win == 512) launch_wmean_seg<512>(logl, grid, blk, st, S, cols, p1, gp, (unsigned*)workspace);
  else if (win == 256) launch_wmean_seg<256>(logl, grid, blk, st, S, cols, p1, gp, (unsigned*)workspace);
  else launch_wmean_seg<128>(logl, grid, blk, st, S, cols, p1, gp, (unsigned*)workspace);
  return launch_err();
}

int qz_awq_stats_layout(int32_t which, int64_t rows, int64_t cols, int32_t group_size, int64_t* out) {
  if (!out) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0 || (which != 0 && which != 1) || (which == 1 && group_size <= 0)) return QZ_ERR_SHAPE;
  int64_t rc = 0, nch = 0;
  const int64_t n1 = which == 0 ? absmean_1l(rows, cols, &rc) : wmean_1l(rows, cols, group_size, &rc);
  int win = 512, swp = which == 0 ? AWP : WWP, tf = FW;
  int64_t cpg = 0;
  if (n1 > 0) {
    nch = n1;
    win = which == 0 ? ABS1_WIN : wmean_win(group_size);
    swp = which == 0 ? ABS1_SWP : WM1_SWP;
    tf = swp * 64 / win;
    cpg = QZ_STATS_CPG;
  } else {
    nch = which == 0 ? absmean_chunks(rows, cols, &rc) : wmean_chunks(rows, cols, &rc);
  }
  out[0] = n1 > 0;
  out[1] = win;
  out[2] = rc;
  out[3] = nch;
  out[4] = (int64_t)swp * 64 / (win / 8);  // row slots per workgroup
  out[5] = tf;
  out[6] = n1 > 0 ? STATS_HEAD : 0;
  out[7] = cpg;  // chunks per first-level group (0: the two-launch plan)
  return QZ_OK;
}

int qz_awq_grid_scales(const float* x_mean, const float* w_mean, int64_t channels, float ratio, int32_t duo_scaling,
                       float* scales_out, qz_stream_t stream) {
  if (!x_mean || !scales_out || (duo_scaling && !w_mean)) return QZ_ERR_NULL;
  if (channels <= 0 || channels > 65536) return QZ_ERR_SHAPE;
  hipLaunchKernelGGL(k_grid_scales, dim3(1), dim3(1024), 0, (hipStream_t)stream, x_mean, w_mean, channels, ratio,
                     (int)duo_scaling, scales_out);
  return launch_err();
}

int qz_awq_grid_scales_batched(const float* x_mean, const float* w_mean, int64_t batch, int64_t channels,
                               float ratio, int32_t duo_scaling, float* scales_out, qz_stream_t stream) {
  if (!x_mean || !scales_out || (duo_scaling && !w_mean)) return QZ_ERR_NULL;
  if (channels <= 0 || channels > 65536 || batch <= 0 || batch > 65535) return QZ_ERR_SHAPE;
  hipLaunchKernelGGL(k_grid_scales, dim3((unsigned)batch), dim3(1024), 0, (hipStream_t)stream, x_mean, w_mean,
                     channels, ratio, (int)duo_scaling, scales_out);
  return launch_err();
}

int qz_scale_columns(void* w, int64_t rows, int64_t cols, int64_t ld, const float* s, int32_t divide,
                     qz_stream_t stream) {
  if (!w || !s) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0 || ld < cols) return QZ_ERR_SHAPE;
  if (v8_ok(w, cols, ld, s, true)) {
    dim3 grid((unsigned)cdiv(cols / 8, 256), (unsigned)std::min<int64_t>(rows, 65535));
    hipLaunchKernelGGL(k_scale_v8<true>, grid, dim3(256), 0, (hipStream_t)stream, (uint16_t*)w, rows, cols, ld, s,
                       (int)divide);
    return launch_err();
  }
  hipLaunchKernelGGL(k_scale_cols, dim3((unsigned)cdiv(rows * cols, 256)), dim3(256), 0, (hipStream_t)stream,
                     (uint16_t*)w, rows, cols, ld, s, (int)divide);
  return launch_err();
}

int qz_scale_rows(void* w, int64_t rows, int64_t cols, int64_t ld, const float* s, int32_t divide,
                  qz_stream_t stream) {
  if (!w || !s) return QZ_ERR_NULL;
  if (rows <= 0 || cols <= 0 || ld < cols) return QZ_ERR_SHAPE;
  if (v8_ok(w, cols, ld, s, false)) {
    dim3 grid((unsigned)cdiv(cols / 8, 256), (unsigned)std::min<int64_t>(rows, 65535));
    hipLaunchKernelGGL(k_scale_v8<false>, grid, dim3(256), 0, (hipStream_t)stream, (uint16_t*)w, rows, cols, ld, s,
                       (int)divide);
    return launch_err();
  }
  hipLaunchKernelGGL(k_scale_rows, dim3((unsigned)cdiv(rows * cols, 256)), dim3(256), 0, (hipStream_t)stream,
                     (uint16_t*)w, rows, cols, ld, s, (int)divide);
  return launch_err();
}

}  // extern "C"
