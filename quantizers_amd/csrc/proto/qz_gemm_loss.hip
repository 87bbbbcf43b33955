// Prototype: the AWQ expert search's grid-point loss
//   loss_i = sum_{t,n} f32(bf16(bf16(X_i W_i^T)[t,n] - R_i[t,n]))^2
// for a batch of items i (experts x grid points): X_i [T_i, K] bf16 (an expert's inputs), W_i [N, K]
// bf16 (its fake-quantized w2 at one grid point), R_i [T_i, N] bf16 (its reference output), fused into
// ONE MFMA launch: no [T, N] output round trip, no separate loss pass.
//
// Structure: 256 x 256 output tile per 512-thread workgroup (8 waves, 2 (t) x 4 (n), 128 x 64 per
// wave, 8 x 4 accumulators of mfma_f32_16x16x32_bf16), K in steps of 32 through a 4-stage LDS ring
// (A 16 KB + B 16 KB per stage) filled by global_load_lds_dwordx4 two steps ahead, counted vmcnt and
// a raw s_barrier per step; LDS rows of 64 B with the 16-B chunk index XORed with sw32(row) so
// each lane group of a wave's ds_read_b128 of a fragment touches every bank once.  grid = (tiles, items); the
// workgroups of one item's t-row of tiles share an XCD (bijective remap).  Rows past T_i are loaded
// as row T_i - 1 and skipped by the epilogue.  Each workgroup writes ONE f64 partial (0 for a tile
// past its item's rows): part_i[tile], summed by the caller in a fixed order.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace {
constexpr int BM = 256, BN = 256, BK = 32, NST = 4, NTH = 512;
constexpr int STAGE_A = BM * BK * 2;            // 16 KB
constexpr int STAGE = STAGE_A + BN * BK * 2;    // 32 KB
constexpr int LDS_BYTES = NST * STAGE;          // 128 KB

__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }

// BK 32 layout: 16-B chunk c of row r at physical chunk c ^ sw32(r), sw32 = (0, 2, 3, 1)[(r >> 2) & 3]:
// with 64-B rows four rows share a 256-B bank row, and gfx950 services a ds_read_b128 in the lane
// groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} (+32): a fragment read (row = lane & 15, chunk =
// lane >> 4) puts each group on 16 distinct 16-B bank slots (the round-6 first build's (r >> 2) & 3
// was 2-way in every group; MI355X_MICROARCH.md §LDS)
__device__ __forceinline__ int sw32(int row) { return (0x78 >> (2 * ((row >> 2) & 3))) & 3; }

// one stage: rows [r0, r0 + 256) (clamped to rmax - 1) of a K-contiguous operand, columns
// [k0, k0 + 32), into the LDS region at `dst` (row r at dst + 64 r, chunk c at c ^ sw32(r))
__device__ __forceinline__ void stage_rows(const uint16_t* __restrict__ src, int64_t ld, int64_t r0, int64_t rmax,
                                           int64_t k0, uint8_t* dst, int w, int lane) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int R = (w * 2 + q) * 16;  // this wave-instruction's first row (16 rows x 64 B = 1 KB)
    const int row = R + (lane >> 2);
    const int c = (lane & 3) ^ sw32(row);
    const int64_t gr = r0 + row < rmax ? r0 + row : rmax - 1;
    const uint16_t* g = src + gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(dst + R * 64), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag_c(const uint8_t* base, int row, int chunk) {
  const int c = chunk ^ sw32(row);
  return *reinterpret_cast<const bf16x8*>(base + row * 64 + c * 16);
}

struct Item {  // one (expert, grid point): device table row of 5 x 8 bytes
  const uint16_t* x;
  const uint16_t* w;
  const uint16_t* r;
  double* part;
  int64_t rows;
};

// one stage of BK64: 256 rows x 128 B, chunk c of row r at physical chunk c ^ ((r >> 1) & 7)
__device__ __forceinline__ void stage_rows64(const uint16_t* __restrict__ src, int64_t ld, int64_t r0, int64_t rmax,
                                             int64_t k0, uint8_t* dst, int w, int lane) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int R = (w * 4 + q) * 8;  // this wave-instruction's first row (8 rows x 128 B = 1 KB)
    const int row = R + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int64_t gr = r0 + row < rmax ? r0 + row : rmax - 1;
    const uint16_t* g = src + gr * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(dst + R * 128), 16, 0, 0);
  }
}
__device__ __forceinline__ bf16x8 frag64(const uint8_t* base, int row, int chunk) {
  const int c = chunk ^ ((row >> 1) & 7);
  return *reinterpret_cast<const bf16x8*>(base + row * 128 + c * 16);
}

// TRANS: the product computed as (W X^T) so each lane's 4 accumulator registers are 4 consecutive
// n of one t (R read 8 bytes at a time); else X W^T (registers = 4 consecutive t of one n).
template <int MODE, bool TRANS>  // MODE 0: store bf16 C (testing); 1: loss partials
__global__ __launch_bounds__(NTH) void k_gemm_sqerr(const Item* __restrict__ items, uint16_t* __restrict__ C, int64_t N,
                                                    int64_t K, int64_t tiles_max) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const Item it = items[blockIdx.y];
  const int ntn = (int)(N / BN);
  const int64_t tiles = (it.rows + BM - 1) / BM * ntn;
  // bijective XCD remap over tiles_max workgroups: consecutive tile ids share an XCD
  const int64_t b = blockIdx.x, xcd = b & 7, q8 = tiles_max >> 3, r8 = tiles_max & 7;
  const int64_t idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  if (idx >= tiles) {  // past this item's rows: a zero partial keeps the fixed-order sum dense
    if (MODE == 1 && tid == 0) it.part[idx] = 0.0;
    return;
  }
  const int64_t t0 = idx / ntn * BM, n0 = idx % ntn * BN;
  const int nk = (int)(K / BK);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  stage_rows(it.x, K, t0, it.rows, 0, lds, w, lane);
  stage_rows(it.w, K, n0, N, 0, lds + STAGE_A, w, lane);
  if (nk > 1) {
    stage_rows(it.x, K, t0, it.rows, BK, lds + STAGE, w, lane);
    stage_rows(it.w, K, n0, N, BK, lds + STAGE + STAGE_A, w, lane);
  }
  for (int s = 0; s < nk; ++s) {
    if (s + 2 < nk) {
      uint8_t* st = lds + ((s + 2) & (NST - 1)) * STAGE;
      stage_rows(it.x, K, t0, it.rows, (int64_t)(s + 2) * BK, st, w, lane);
      stage_rows(it.w, K, n0, N, (int64_t)(s + 2) * BK, st + STAGE_A, w, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (s + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const uint8_t* st = lds + (s & (NST - 1)) * STAGE;
    bf16x8 xa[8], wb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wb[j] = frag_c(st + STAGE_A, wn * 64 + j * 16 + (lane & 15), lane >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) xa[i] = frag_c(st, wm * 128 + i * 16 + (lane & 15), lane >> 4);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = TRANS ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j], xa[i], acc[i][j], 0, 0, 0)
                          : __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[i], wb[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  }

  // epilogue.  16x16x32 C/D: col = lane & 15, row = (lane >> 4) * 4 + reg.  X W^T: col = n, row = t;
  // W X^T: col = t, row = n.
  double dsum = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (TRANS) {
        const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
        const int64_t n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
        if (t >= it.rows) continue;
        if constexpr (MODE == 0) {
          *reinterpret_cast<uint2*>(C + t * N + n) = make_uint2(lo, hi);
        } else {
          const uint2 rv = *reinterpret_cast<const uint2*>(it.r + t * N + n);
          const float d0 = bf2f(f2bf(bf2f(lo & 0xffffu) - bf2f(rv.x & 0xffffu)));
          const float d1 = bf2f(f2bf(bf2f(lo >> 16) - bf2f(rv.x >> 16)));
          const float d2 = bf2f(f2bf(bf2f(hi & 0xffffu) - bf2f(rv.y & 0xffffu)));
          const float d3 = bf2f(f2bf(bf2f(hi >> 16) - bf2f(rv.y >> 16)));
          dsum += (double)(d0 * d0 + d1 * d1) + (double)(d2 * d2 + d3 * d3);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t t = t0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
          const int64_t n = n0 + wn * 64 + j * 16 + (lane & 15);
          if (t >= it.rows) continue;
          const uint16_t o = f2bf(acc[i][j][r]);
          if constexpr (MODE == 0) {
            C[t * N + n] = o;
          } else {
            const float d = bf2f(f2bf(bf2f(o) - bf2f(it.r[t * N + n])));
            dsum += (double)(d * d);
          }
        }
      }
    }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dsum += __shfl_xor(dsum, off);
    double* wsum = reinterpret_cast<double*>(lds);  // the ring is free: one __shared__ object only
    __syncthreads();
    if (lane == 0) wsum[w] = dsum;
    __syncthreads();
    if (tid == 0) {
      double tt = 0;
      for (int i = 0; i < 8; ++i) tt += wsum[i];
      it.part[idx] = tt;
    }
  }
}
// TRANS: the product computed as (W X^T) so each lane's 4 accumulator registers are 4 consecutive
// n of one t (R read 8 bytes at a time); else X W^T (registers = 4 consecutive t of one n).
template <int MODE, bool TRANS>  // MODE 0: store bf16 C (testing); 1: loss partials
__global__ __launch_bounds__(NTH) void k_gemm_sqerr64(const Item* __restrict__ items, uint16_t* __restrict__ C, int64_t N,
                                                    int64_t K, int64_t tiles_max) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const Item it = items[blockIdx.y];
  const int ntn = (int)(N / BN);
  const int64_t tiles = (it.rows + BM - 1) / BM * ntn;
  // bijective XCD remap over tiles_max workgroups: consecutive tile ids share an XCD
  const int64_t b = blockIdx.x, xcd = b & 7, q8 = tiles_max >> 3, r8 = tiles_max & 7;
  const int64_t idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  if (idx >= tiles) {  // past this item's rows: a zero partial keeps the fixed-order sum dense
    if (MODE == 1 && tid == 0) it.part[idx] = 0.0;
    return;
  }
  const int64_t t0 = idx / ntn * BM, n0 = idx % ntn * BN;
  const int nk = (int)(K / BK);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // BK = 64, two 64 KB stages: step s + 1 is issued right after step s's barrier (its stage was
  // last read at step s - 1) and lands during step s's MFMAs
  constexpr int BK2 = 64, ST2 = 65536, ST2A = 32768;
  const int nk2 = (int)(K / BK2);
  // per-lane source rows of this workgroup's 4 + 4 wave-instructions, fixed for the tile
  const uint16_t* gx[4];
  const uint16_t* gw[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int row = (w * 4 + q) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int64_t rx = t0 + row < it.rows ? t0 + row : it.rows - 1;
    gx[q] = it.x + rx * K + c * 8;
    gw[q] = it.w + (n0 + row) * K + c * 8;
  }
  auto stage64 = [&](int s, uint8_t* dst) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      __builtin_amdgcn_global_load_lds((const void*)(gx[q] + s * BK2),
                                       (__attribute__((address_space(3))) void*)(dst + (w * 4 + q) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(gw[q] + s * BK2),
                                       (__attribute__((address_space(3))) void*)(dst + ST2A + (w * 4 + q) * 1024), 16,
                                       0, 0);
    }
  };
  stage64(0, lds);
  for (int s = 0; s < nk2; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nk2) stage64(s + 1, lds + ((s + 1) & 1) * ST2);
    const uint8_t* st = lds + (s & 1) * ST2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 xa[8], wb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) wb[j] = frag64(st + ST2A, wn * 64 + j * 16 + (lane & 15), ks * 4 + (lane >> 4));
#pragma unroll
      for (int i = 0; i < 8; ++i) xa[i] = frag64(st, wm * 128 + i * 16 + (lane & 15), ks * 4 + (lane >> 4));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = TRANS ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j], xa[i], acc[i][j], 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_bf16(xa[i], wb[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }

  // epilogue.  16x16x32 C/D: col = lane & 15, row = (lane >> 4) * 4 + reg.  X W^T: col = n, row = t;
  // W X^T: col = t, row = n.
  double dsum = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if constexpr (TRANS) {
        const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
        const int64_t n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
        if (t >= it.rows) continue;
        if constexpr (MODE == 0) {
          *reinterpret_cast<uint2*>(C + t * N + n) = make_uint2(lo, hi);
        } else {
          const uint2 rv = *reinterpret_cast<const uint2*>(it.r + t * N + n);
          const float d0 = bf2f(f2bf(bf2f(lo & 0xffffu) - bf2f(rv.x & 0xffffu)));
          const float d1 = bf2f(f2bf(bf2f(lo >> 16) - bf2f(rv.x >> 16)));
          const float d2 = bf2f(f2bf(bf2f(hi & 0xffffu) - bf2f(rv.y & 0xffffu)));
          const float d3 = bf2f(f2bf(bf2f(hi >> 16) - bf2f(rv.y >> 16)));
          dsum += (double)(d0 * d0 + d1 * d1) + (double)(d2 * d2 + d3 * d3);
        }
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t t = t0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
          const int64_t n = n0 + wn * 64 + j * 16 + (lane & 15);
          if (t >= it.rows) continue;
          const uint16_t o = f2bf(acc[i][j][r]);
          if constexpr (MODE == 0) {
            C[t * N + n] = o;
          } else {
            const float d = bf2f(f2bf(bf2f(o) - bf2f(it.r[t * N + n])));
            dsum += (double)(d * d);
          }
        }
      }
    }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dsum += __shfl_xor(dsum, off);
    double* wsum = reinterpret_cast<double*>(lds);  // the ring is free: one __shared__ object only
    __syncthreads();
    if (lane == 0) wsum[w] = dsum;
    __syncthreads();
    if (tid == 0) {
      double tt = 0;
      for (int i = 0; i < 8; ++i) tt += wsum[i];
      it.part[idx] = tt;
    }
  }
}

// 4-wave variant (hipBLASLt's MT256x256x64 / MI16x16 shape, profiles/r06n_gemm_pmc.txt): 256-thread
// workgroups, 2 x 2 waves of 128 (t) x 128 (n), 8 x 8 accumulators (256 registers, one wave per
// SIMD), BK = 64 through two 64 KB stages; 2 x 8 fragments per k-substep, so a third fewer LDS
// reads per MFMA than the 8-wave form.
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_gemm_sqerr4w(const Item* __restrict__ items, uint16_t* __restrict__ C, int64_t N, int64_t K, int64_t tiles_max) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const Item it = items[blockIdx.y];
  const int ntn = (int)(N / BN);
  const int64_t tiles = (it.rows + BM - 1) / BM * ntn;
  const int64_t b = blockIdx.x, xcd = b & 7, q8 = tiles_max >> 3, r8 = tiles_max & 7;
  const int64_t idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  if (idx >= tiles) {
    if (MODE == 1 && tid == 0) it.part[idx] = 0.0;
    return;
  }
  const int64_t t0 = idx / ntn * BM, n0 = idx % ntn * BN;
  constexpr int BK2 = 64, ST2 = 65536, ST2A = 32768;
  const int nk2 = (int)(K / BK2);
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // wave w stages rows [w * 64, w * 64 + 64) of both operands: 8 wave-instructions of 8 rows each
  const int row0 = w * 64 + (lane >> 3);
  const int c0 = lane & 7;
  auto stage64 = [&](int s, uint8_t* dst) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int row = row0 + q * 8;
      const int c = c0 ^ ((row >> 1) & 7);
      const int64_t rx = t0 + row < it.rows ? t0 + row : it.rows - 1;
      __builtin_amdgcn_global_load_lds((const void*)(it.x + rx * K + (int64_t)s * BK2 + c * 8),
                                       (__attribute__((address_space(3))) void*)(dst + (w * 8 + q) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(it.w + (n0 + row) * K + (int64_t)s * BK2 + c * 8),
                                       (__attribute__((address_space(3))) void*)(dst + ST2A + (w * 8 + q) * 1024), 16,
                                       0, 0);
    }
  };
  stage64(0, lds);
  for (int s = 0; s < nk2; ++s) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 1 < nk2) stage64(s + 1, lds + ((s + 1) & 1) * ST2);
    const uint8_t* st = lds + (s & 1) * ST2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      bf16x8 xa[8], wb[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) wb[j] = frag64(st + ST2A, wn * 128 + j * 16 + (lane & 15), ks * 4 + (lane >> 4));
#pragma unroll
      for (int i = 0; i < 8; ++i) xa[i] = frag64(st, wm * 128 + i * 16 + (lane & 15), ks * 4 + (lane >> 4));
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j], xa[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  double dsum = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
      const int64_t n = n0 + wn * 128 + j * 16 + (lane >> 4) * 4;
      const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
      const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
      if (t >= it.rows) continue;
      if constexpr (MODE == 0) {
        *reinterpret_cast<uint2*>(C + t * N + n) = make_uint2(lo, hi);
      } else {
        const uint2 rv = *reinterpret_cast<const uint2*>(it.r + t * N + n);
        const float d0 = bf2f(f2bf(bf2f(lo & 0xffffu) - bf2f(rv.x & 0xffffu)));
        const float d1 = bf2f(f2bf(bf2f(lo >> 16) - bf2f(rv.x >> 16)));
        const float d2 = bf2f(f2bf(bf2f(hi & 0xffffu) - bf2f(rv.y & 0xffffu)));
        const float d3 = bf2f(f2bf(bf2f(hi >> 16) - bf2f(rv.y >> 16)));
        dsum += (double)(d0 * d0 + d1 * d1) + (double)(d2 * d2 + d3 * d3);
      }
    }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dsum += __shfl_xor(dsum, off);
    double* wsum = reinterpret_cast<double*>(lds);
    __syncthreads();
    if (lane == 0) wsum[w] = dsum;
    __syncthreads();
    if (tid == 0) it.part[idx] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
  }
}

// 4-wave software-pipelined variant: the fragments of the next k-substep are read (16 ds_read_b128)
// while the 64 MFMAs of the current one issue, interleaved 1 : 4 by sched_group_barrier; two
// fragment register sets; one barrier per 64-deep step, after which the glds for step s + 2 go into
// the stage just drained.
struct Frag16 {
  bf16x8 x[8], w[8];
};
__device__ __forceinline__ void load_frags(Frag16& f, const uint8_t* st, int wm, int wn, int ks, int lane) {
#pragma unroll
  for (int j = 0; j < 8; ++j) f.w[j] = frag64(st + 32768, wn * 128 + j * 16 + (lane & 15), ks * 4 + (lane >> 4));
#pragma unroll
  for (int i = 0; i < 8; ++i) f.x[i] = frag64(st, wm * 128 + i * 16 + (lane & 15), ks * 4 + (lane >> 4));
}
__device__ __forceinline__ void mma_all(f32x4 (&acc)[8][8], const Frag16& f) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.w[j], f.x[i], acc[i][j], 0, 0, 0);
}
__device__ __forceinline__ void interleave_16r_64m() {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // 1 DS read
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);  // 4 MFMA
  }
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_gemm_sqerr4p(const Item* __restrict__ items, uint16_t* __restrict__ C, int64_t N, int64_t K, int64_t tiles_max) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  const Item it = items[blockIdx.y];
  const int ntn = (int)(N / BN);
  const int64_t tiles = (it.rows + BM - 1) / BM * ntn;
  const int64_t b = blockIdx.x, xcd = b & 7, q8 = tiles_max >> 3, r8 = tiles_max & 7;
  const int64_t idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  if (idx >= tiles) {
    if (MODE == 1 && tid == 0) it.part[idx] = 0.0;
    return;
  }
  const int64_t t0 = idx / ntn * BM, n0 = idx % ntn * BN;
  constexpr int BK2 = 64, ST2 = 65536, ST2A = 32768;
  const int nk2 = (int)(K / BK2);
  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint16_t* gx[8];
  const uint16_t* gw[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int row = w * 64 + q * 8 + (lane >> 3);
    const int c = (lane & 7) ^ ((row >> 1) & 7);
    const int64_t rx = t0 + row < it.rows ? t0 + row : it.rows - 1;
    gx[q] = it.x + rx * K + c * 8;
    gw[q] = it.w + (n0 + row) * K + c * 8;
  }
  auto stage64 = [&](int s, uint8_t* dst) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      __builtin_amdgcn_global_load_lds((const void*)(gx[q] + s * BK2),
                                       (__attribute__((address_space(3))) void*)(dst + (w * 8 + q) * 1024), 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const void*)(gw[q] + s * BK2),
                                       (__attribute__((address_space(3))) void*)(dst + ST2A + (w * 8 + q) * 1024), 16,
                                       0, 0);
    }
  };
  Frag16 f0, f1;
  stage64(0, lds);
  if (nk2 > 1) stage64(1, lds + ST2);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // step 0 (this wave's 16 loads) landed
  __builtin_amdgcn_s_barrier();
  load_frags(f0, lds, wm, wn, 0, lane);
  for (int s = 0; s < nk2; ++s) {
    const uint8_t* st = lds + (s & 1) * ST2;
    // half 1: read (s, ks 1) while the MFMAs of (s, ks 0) issue
    load_frags(f1, st, wm, wn, 1, lane);
    mma_all(acc, f0);
    interleave_16r_64m();
    // every wave has read stage s; step s + 1 landed: barrier, then refill stage s with step s + 2
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (s + 2 < nk2) stage64(s + 2, lds + (s & 1) * ST2);
    // half 2: read (s + 1, ks 0) while the MFMAs of (s, ks 1) issue
    if (s + 1 < nk2) load_frags(f0, lds + ((s + 1) & 1) * ST2, wm, wn, 0, lane);
    mma_all(acc, f1);
    interleave_16r_64m();
  }
  double dsum = 0.0;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
      const int64_t n = n0 + wn * 128 + j * 16 + (lane >> 4) * 4;
      const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
      const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
      if (t >= it.rows) continue;
      if constexpr (MODE == 0) {
        *reinterpret_cast<uint2*>(C + t * N + n) = make_uint2(lo, hi);
      } else {
        const uint2 rv = *reinterpret_cast<const uint2*>(it.r + t * N + n);
        const float d0 = bf2f(f2bf(bf2f(lo & 0xffffu) - bf2f(rv.x & 0xffffu)));
        const float d1 = bf2f(f2bf(bf2f(lo >> 16) - bf2f(rv.x >> 16)));
        const float d2 = bf2f(f2bf(bf2f(hi & 0xffffu) - bf2f(rv.y & 0xffffu)));
        const float d3 = bf2f(f2bf(bf2f(hi >> 16) - bf2f(rv.y >> 16)));
        dsum += (double)(d0 * d0 + d1 * d1) + (double)(d2 * d2 + d3 * d3);
      }
    }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dsum += __shfl_xor(dsum, off);
    double* wsum = reinterpret_cast<double*>(lds);
    __syncthreads();
    if (lane == 0) wsum[w] = dsum;
    __syncthreads();
    if (tid == 0) it.part[idx] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
  }
}

// Staggered-phase variant (round 6, after VERDICT r05's stop: the guide's 256^2 8-phase schedule recast
// for BK 32 and this kernel's 4-stage ring).  8 waves of 128 (t) x 64 (n) as k_gemm_sqerr<.., true>;
// each K step is two phases of 16 MFMAs (the wave's t rows 0-63, then 64-127).  Phase p:
//   its fragment reads (8, then 4: the W fragments stay for the second phase);
//   half h = p + 5 of the load stream (step h >> 1; X if h is even, W if odd; 2 glds per lane);
//   [second phase of a step: counted vmcnt retiring the next step];
//   s_barrier; lgkmcnt(0); setprio 1; 16 MFMAs; setprio 0; s_barrier.
// Waves 4-7 run one barrier behind waves 0-3 (an extra s_barrier at the start, matched by waves 0-3 at
// the end), so each SIMD's two waves alternate: one issues MFMAs while the other reads and stages.
// Barrier arithmetic (a wave of 4-7's first barrier of phase p IS the second barrier of phase p of
// waves 0-3): data retired by the waits of phase p is read from phase p + 1 on by both groups, and a
// stage last read in phase q may be restaged from phase q + 2 on -- step u's X half is staged in
// phase 2u - 5 and its W half in 2u - 4, while step u - 4, the stage's previous content, was last read
// in phase 2u - 7.
__device__ __forceinline__ void bar_fenced() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int MODE>
__global__ __launch_bounds__(NTH) void k_gemm_sqerr8s(const Item* __restrict__ items, uint16_t* __restrict__ C,
                                                      int64_t N, int64_t K, int64_t tiles_max) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const Item it = items[blockIdx.y];
  const int ntn = (int)(N / BN);
  const int64_t tiles = (it.rows + BM - 1) / BM * ntn;
  const int64_t b = blockIdx.x, xcd = b & 7, q8 = tiles_max >> 3, r8 = tiles_max & 7;
  const int64_t idx = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  if (idx >= tiles) {
    if (MODE == 1 && tid == 0) it.part[idx] = 0.0;
    return;
  }
  const int64_t t0 = idx / ntn * BM, n0 = idx % ntn * BN;
  const int nk = (int)(K / BK), nh = 2 * nk;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // this lane's sources for its wave's 2 instructions of a half (stage_rows' layout)
  const uint16_t* gx[2];
  const uint16_t* gw[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int row = (w * 2 + q) * 16 + (lane >> 2);
    const int c = (lane & 3) ^ sw32(row);
    const int64_t rx = t0 + row < it.rows ? t0 + row : it.rows - 1;
    gx[q] = it.x + rx * K + c * 8;
    gw[q] = it.w + (n0 + row) * K + c * 8;
  }
  auto stage_half = [&](int h) {
    const int u = h >> 1;
    uint8_t* dst = lds + (u & (NST - 1)) * STAGE + (h & 1) * STAGE_A;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const uint16_t* src = ((h & 1) ? gw[q] : gx[q]) + (int64_t)u * BK;
      __builtin_amdgcn_global_load_lds((const void*)src,
                                       (__attribute__((address_space(3))) void*)(dst + (w * 2 + q) * 1024), 16, 0, 0);
    }
  };
  // the halves issued after h0 - 1 may stay in flight: 2 glds each
  auto wait_upto = [&](int h0) {
    const int out = (h0 < nh ? 1 : 0) + (h0 + 1 < nh ? 1 : 0) + (h0 + 2 < nh ? 1 : 0);
    if (out == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (out == 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (out == 1) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  for (int h = 0; h < 5 && h < nh; ++h) stage_half(h);
  wait_upto(2);  // step 0 landed
  bar_fenced();
  if (wm == 1) bar_fenced();  // the stagger
  for (int s = 0; s < nk; ++s) {
    const uint8_t* st = lds + (s & (NST - 1)) * STAGE;
    bf16x8 xa[4], wb[4];
    // phase 2s: t rows 0-63 of the wave
#pragma unroll
    for (int j = 0; j < 4; ++j) wb[j] = frag_c(st + STAGE_A, wn * 64 + j * 16 + (lane & 15), lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[i] = frag_c(st, wm * 128 + i * 16 + (lane & 15), lane >> 4);
    if (2 * s + 5 < nh) stage_half(2 * s + 5);
    bar_fenced();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j], xa[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar_fenced();
    // phase 2s + 1: t rows 64-127
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[i] = frag_c(st, wm * 128 + (4 + i) * 16 + (lane & 15), lane >> 4);
    if (2 * s + 6 < nh) stage_half(2 * s + 6);
    wait_upto(2 * s + 4);  // step s + 1 (halves 2s + 2, 2s + 3) landed
    bar_fenced();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j], xa[i], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar_fenced();
  }
  if (wm == 0) bar_fenced();  // matches waves 4-7's extra barrier

  double dsum = 0.0;
  if constexpr (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
        const int64_t n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
        if (t < it.rows) *reinterpret_cast<uint2*>(C + t * N + n) = make_uint2(lo, hi);
      }
  } else {
    // every R load of the lane issued before the first use (rows past the item's clamped, masked)
    uint2 rv[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
        const int64_t tc = t < it.rows ? t : it.rows - 1;
        rv[i][j] = *reinterpret_cast<const uint2*>(it.r + tc * N + n0 + wn * 64 + j * 16 + (lane >> 4) * 4);
      }
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
        const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
        const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
        const float d0 = bf2f(f2bf(bf2f(lo & 0xffffu) - bf2f(rv[i][j].x & 0xffffu)));
        const float d1 = bf2f(f2bf(bf2f(lo >> 16) - bf2f(rv[i][j].x >> 16)));
        const float d2 = bf2f(f2bf(bf2f(hi & 0xffffu) - bf2f(rv[i][j].y & 0xffffu)));
        const float d3 = bf2f(f2bf(bf2f(hi >> 16) - bf2f(rv[i][j].y >> 16)));
        if (t < it.rows) dsum += (double)(d0 * d0 + d1 * d1) + (double)(d2 * d2 + d3 * d3);
      }
  }
  if constexpr (MODE == 1) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) dsum += __shfl_xor(dsum, off);
    double* wsum = reinterpret_cast<double*>(lds);
    __syncthreads();
    if (lane == 0) wsum[w] = dsum;
    __syncthreads();
    if (tid == 0) {
      double tt = 0;
      for (int i = 0; i < 8; ++i) tt += wsum[i];
      it.part[idx] = tt;
    }
  }
}

// Persistent form of k_gemm_sqerr8s (round 6): one workgroup per CU walks its tiles (global tile G = k
// * gridDim.x + slot over all items, slot the bijective XCD remap, so an XCD's workgroups share each
// X row-block) and the load stream never stops at a tile boundary: phase p of the walk issues half p
// + 5 of the stream (the next tile's first steps land under this tile's last MFMAs), and a stream past
// the walk's last tile keeps issuing into a spare 16 KB of LDS so every counted vmcnt is a constant.
// R's 32 values per lane are loaded in the first phase of step nk - 2 (two vmcnt windows then allow 32
// more), so the loss epilogue finds them in registers; with the stagger one group's epilogue runs
// under the other group's MFMAs.  Partials per wave: part[idx * 8 + wave] (fixed order for the caller).
template <int MODE>
__global__ __launch_bounds__(NTH) void k_gemm_sqerr8p(const Item* __restrict__ items, uint16_t* __restrict__ C,
                                                      int64_t N, int64_t K, int tiles_max, int n_items) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES + 16384];
  uint8_t* const spare = lds + LDS_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = (int)(N / BN), nk = (int)(K / BK);
  const int nwg = (int)gridDim.x, b = (int)blockIdx.x, xcd = b & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int slot = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  // the walk: global tiles slot, slot + nwg, ... as (item, idx) pairs kept in scalar registers (a 64-bit
  // division would leave them in VGPRs, the Item reads would become vector loads, and their vmcnt(0)
  // would drain the load stream at every tile)
  struct Walk {
    int item, idx;
  };
  auto uni = [](int v) { return __builtin_amdgcn_readfirstlane(v); };
  auto step_walk = [&](Walk& p) {
    int idx = p.idx + nwg, item = p.item;
    while (idx >= tiles_max) {
      idx -= tiles_max;
      ++item;
    }
    p.idx = uni(idx);
    p.item = uni(item);
  };
  // the item table through the constant address space: scalar loads (the stores to `part` would
  // otherwise keep the compiler from proving it unclobbered, and it would read it with vector loads)
  typedef const __attribute__((address_space(4))) Item CItem;
  CItem* const citems = (CItem*)items;
  auto item_at = [&](int i) {
    Item r;
    r.x = citems[i].x;
    r.w = citems[i].w;
    r.r = citems[i].r;
    r.part = citems[i].part;
    r.rows = citems[i].rows;
    return r;
  };
  auto tiles_of = [&](int it) { return (int)((citems[it].rows + BM - 1) / BM) * ntn; };
  auto valid = [&](const Walk& p) { return p.item < n_items && p.idx < tiles_of(p.item); };
  const Walk first = {uni(slot / tiles_max), uni(slot % tiles_max)};

  // ---- the load stream
  Walk sw = first;
  while (sw.item < n_items && !valid(sw)) step_walk(sw);
  bool live = sw.item < n_items;
  const uint16_t* gx[2];
  const uint16_t* gw[2];
  auto set_ptrs = [&](const Walk& p) {
    const Item it = item_at(p.item);
    const int64_t t0 = (int64_t)(p.idx / ntn) * BM, n0 = (int64_t)(p.idx % ntn) * BN;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int row = (w * 2 + q) * 16 + (lane >> 2);
      const int c = (lane & 3) ^ sw32(row);
      const int64_t rx = t0 + row < it.rows ? t0 + row : it.rows - 1;
      gx[q] = it.x + rx * K + c * 8;
      gw[q] = it.w + (n0 + row) * K + c * 8;
    }
  };
  if (!live) {  // nothing valid for this workgroup: zero partials only
    if (MODE == 1 && lane == 0)
      for (Walk p = first; p.item < n_items; step_walk(p)) item_at(p.item).part[(int64_t)p.idx * 8 + w] = 0.0;
    return;
  }
  set_ptrs(sw);
  int us = 0, ps = 0;
  int64_t gs = 0;
  auto issue = [&]() {
    if (live) {
      uint8_t* dst = lds + (gs & (NST - 1)) * STAGE + ps * STAGE_A;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds((const void*)((ps ? gw[q] : gx[q]) + (int64_t)us * BK),
                                         (__attribute__((address_space(3))) void*)(dst + (w * 2 + q) * 1024), 16, 0, 0);
      if (ps) {
        ps = 0;
        ++gs;
        if (++us == nk) {
          us = 0;
          do step_walk(sw);
          while (sw.item < n_items && !valid(sw));
          live = sw.item < n_items;
          if (live) set_ptrs(sw);
        }
      } else {
        ps = 1;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q)
        __builtin_amdgcn_global_load_lds((const void*)gx[q],
                                         (__attribute__((address_space(3))) void*)(spare + (w * 2 + q) * 1024), 16, 0, 0);
    }
  };

  for (int h = 0; h < 5; ++h) issue();
  asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // the walk's first step landed
  bar_fenced();
  if (wm == 1) bar_fenced();  // the stagger

  int64_t gc = 0;  // the walk's global step (its LDS stage: gc & 3)
  f32x4 acc[8][4];
  bf16x8 xa[4], wb[4];
  uint64_t rv[8][4];
  auto phase0 = [&]() {
    const uint8_t* st = lds + (gc & (NST - 1)) * STAGE;
#pragma unroll
    for (int j = 0; j < 4; ++j) wb[j] = frag_c(st + STAGE_A, wn * 64 + j * 16 + (lane & 15), lane >> 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[i] = frag_c(st, wm * 128 + i * 16 + (lane & 15), lane >> 4);
    issue();
  };
  auto mfma0 = [&]() {
    bar_fenced();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j], xa[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar_fenced();
  };
  auto phase1_reads = [&]() {
    const uint8_t* st = lds + (gc & (NST - 1)) * STAGE;
#pragma unroll
    for (int i = 0; i < 4; ++i) xa[i] = frag_c(st, wm * 128 + (4 + i) * 16 + (lane & 15), lane >> 4);
    issue();
  };
  auto mfma1 = [&]() {
    bar_fenced();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[4 + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[j], xa[i], acc[4 + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    bar_fenced();
    ++gc;
  };

  for (Walk cw = first; cw.item < n_items; step_walk(cw)) {
    const Item it = item_at(cw.item);
    const int64_t idx = cw.idx;
    if (cw.idx >= (int)((it.rows + BM - 1) / BM) * ntn) {
      if (MODE == 1 && lane == 0) it.part[idx * 8 + w] = 0.0;
      continue;
    }
    const int64_t t0 = (int64_t)(cw.idx / ntn) * BM, n0 = (int64_t)(cw.idx % ntn) * BN;
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < nk; ++s) {
      phase0();
      mfma0();
      phase1_reads();
      asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // the next step landed
      mfma1();
    }
    // epilogue (runs under the other wave group's MFMAs)
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
          const int64_t n = n0 + wn * 64 + j * 16 + (lane >> 4) * 4;
          const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
          const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
          if (t < it.rows) *reinterpret_cast<uint2*>(C + t * N + n) = make_uint2(lo, hi);
        }
    } else {
      // every R load of the lane first (rows past the item's clamped, masked below)
      const __attribute__((address_space(1))) uint64_t* rg = (const __attribute__((address_space(1))) uint64_t*)it.r;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
          const int64_t tc = t < it.rows ? t : it.rows - 1;
          rv[i][j] = rg[(tc * N + n0 + wn * 64 + j * 16 + (lane >> 4) * 4) >> 2];
        }
      double dsum = 0.0;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t t = t0 + wm * 128 + i * 16 + (lane & 15);
          const uint32_t lo = (uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16);
          const uint32_t hi = (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16);
          const float d0 = bf2f(f2bf(bf2f(lo & 0xffffu) - bf2f((uint32_t)rv[i][j] & 0xffffu)));
          const float d1 = bf2f(f2bf(bf2f(lo >> 16) - bf2f(((uint32_t)rv[i][j] >> 16))));
          const float d2 = bf2f(f2bf(bf2f(hi & 0xffffu) - bf2f((uint32_t)(rv[i][j] >> 32) & 0xffffu)));
          const float d3 = bf2f(f2bf(bf2f(hi >> 16) - bf2f((uint32_t)(rv[i][j] >> 48))));
          if (t < it.rows) dsum += (double)(d0 * d0 + d1 * d1) + (double)(d2 * d2 + d3 * d3);
        }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) dsum += __shfl_xor(dsum, off);
      if (lane == 0) it.part[idx * 8 + w] = dsum;
    }
  }
  if (wm == 0) bar_fenced();  // matches waves 4-7's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stream's last (spare) loads
}
}  // namespace

// items: device array of n Item rows {x, w, r, part, rows}; every item N x K (dense rows: ld = K for
// x and w, N for r); part of item i has tiles_max f64 slots.  mode: bit 0 loss (else store C into
// `C`, item 0 only, testing); bit 1 TRANS; bit 2 BK = 64 with two stages; bit 3 / 4 the 4-wave forms;
// bit 5 the staggered-phase form; bit 6 its persistent form (8 partials per tile: part[idx * 8 + wave]).
extern "C" int64_t qzp_gemm_sqerr_tiles(int64_t rows_max, int64_t N) { return (rows_max + BM - 1) / BM * (N / BN); }

extern "C" int qzp_gemm_sqerr(const void* items, int64_t n, int64_t rows_max, int64_t N, int64_t K, void* C, int mode,
                              void* stream) {
  if (n <= 0 || n > 65535 || N % BN || K % BK || K < BK || rows_max <= 0) return -1;
  const int64_t tiles_max = qzp_gemm_sqerr_tiles(rows_max, N);
  if (tiles_max > 0x7fffffff) return -1;
  typedef void (*KFn)(const Item*, uint16_t*, int64_t, int64_t, int64_t);
  static const KFn fns[8] = {k_gemm_sqerr<0, false>,   k_gemm_sqerr<1, false>,   k_gemm_sqerr<0, true>,
                             k_gemm_sqerr<1, true>,    k_gemm_sqerr64<0, false>, k_gemm_sqerr64<1, false>,
                             k_gemm_sqerr64<0, true>,  k_gemm_sqerr64<1, true>};
  if ((mode & 4) && K % 64) return -1;
  if (mode & 64) {  // the persistent staggered-phase variant: part holds 8 partials per tile
    if (K / BK < 3) return -1;
    int cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      return -1;
    const int64_t total = n * tiles_max, nwg = total < cus ? total : cus;
    if (total > 0x7fffffff) return -1;
    hipLaunchKernelGGL((mode & 1) ? k_gemm_sqerr8p<1> : k_gemm_sqerr8p<0>, dim3((unsigned)nwg), dim3(NTH), 0,
                       (hipStream_t)stream, (const Item*)items, (uint16_t*)C, N, K, (int)tiles_max, (int)n);
    return (int)hipGetLastError();
  }
  if (mode & 32) {  // the staggered-phase variant (BK 32, W X^T orientation)
    hipLaunchKernelGGL((mode & 1) ? k_gemm_sqerr8s<1> : k_gemm_sqerr8s<0>, dim3((unsigned)tiles_max, (unsigned)n),
                       dim3(NTH), 0, (hipStream_t)stream, (const Item*)items, (uint16_t*)C, N, K, tiles_max);
    return (int)hipGetLastError();
  }
  if (mode & 16) {  // the 4-wave software-pipelined variant (BK 64)
    if (K % 64) return -1;
    hipLaunchKernelGGL((mode & 1) ? k_gemm_sqerr4p<1> : k_gemm_sqerr4p<0>, dim3((unsigned)tiles_max, (unsigned)n),
                       dim3(256), 0, (hipStream_t)stream, (const Item*)items, (uint16_t*)C, N, K, tiles_max);
    return (int)hipGetLastError();
  }
  if (mode & 8) {  // the 4-wave variant (BK 64)
    if (K % 64) return -1;
    hipLaunchKernelGGL((mode & 1) ? k_gemm_sqerr4w<1> : k_gemm_sqerr4w<0>, dim3((unsigned)tiles_max, (unsigned)n),
                       dim3(256), 0, (hipStream_t)stream, (const Item*)items, (uint16_t*)C, N, K, tiles_max);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(fns[mode & 7], dim3((unsigned)tiles_max, (unsigned)n), dim3(NTH), 0, (hipStream_t)stream,
                     (const Item*)items, (uint16_t*)C, N, K, tiles_max);
  return (int)hipGetLastError();
}
