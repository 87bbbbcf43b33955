// Prototype: the AWQ expert search's grid-point loss
//   loss = sum_{t,n} f32(bf16(bf16(X W^T)[t,n] - R[t,n]))^2
// for X [T, K] bf16 (an expert's inputs), W [N, K] bf16 (its fake-quantized w2 at one grid point),
// R [T, N] bf16 (the reference output), fused into ONE MFMA kernel: no [T, N] output round trip.
// Step 1 (this file's MODE_STORE): the GEMM core alone, C = bf16(X W^T) stored, to price the MFMA
// structure against hipBLASLt before any epilogue work (kill criterion: DESIGN §12 item 1).
//
// Structure: 256 x 256 output tile per 512-thread workgroup (8 waves, 2 (t) x 4 (n), 128 x 64 per
// wave, 8 x 4 accumulators of mfma_f32_16x16x32_bf16), K in steps of 32 through a 4-stage LDS ring
// (A 16 KB + B 16 KB per stage) filled by global_load_lds_dwordx4 two steps ahead, counted vmcnt and
// a raw s_barrier per step; LDS rows of 64 B with the 16-B chunk index XORed with (row >> 2) & 3 so
// a wave's ds_read_b128 of a fragment touches every bank once.
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {
constexpr int BM = 256, BN = 256, BK = 32, NST = 4, NTH = 512;
constexpr int STAGE_A = BM * BK * 2;            // 16 KB
constexpr int STAGE = STAGE_A + BN * BK * 2;    // 32 KB
constexpr int LDS_BYTES = NST * STAGE;          // 128 KB

__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

// one stage: rows [r0, r0 + 256) of a K-contiguous operand, columns [k0, k0 + 32), into the LDS
// region at `dst` (row r at dst + 64 r, chunk c at physical chunk c ^ ((r >> 2) & 3))
__device__ __forceinline__ void stage_rows(const uint16_t* __restrict__ src, int64_t ld, int64_t r0, int64_t k0,
                                           uint8_t* dst, int w, int lane) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int R = (w * 2 + q) * 16;  // this wave-instruction's first row (16 rows x 64 B = 1 KB)
    const int row = R + (lane >> 2);
    const int c = (lane & 3) ^ ((row >> 2) & 3);
    const uint16_t* g = src + (r0 + row) * ld + k0 + c * 8;
    __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(dst + R * 64), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag_c(const uint8_t* base, int row, int chunk) {
  const int c = chunk ^ ((row >> 2) & 3);
  return *reinterpret_cast<const bf16x8*>(base + row * 64 + c * 16);
}

// SH = 16: mfma_f32_16x16x32_bf16, 8 x 4 accumulators of 4 per wave; SH = 32: mfma_f32_32x32x16_bf16,
// 4 x 2 accumulators of 16 per wave (two k-substeps of 16 per step).  PRIO: s_setprio(1) around the
// MFMA block (guide §5.5 T5).
template <int SH>
struct Acc;
template <>
struct Acc<16> {
  f32x4 v[8][4];
  static constexpr int MI = 8, NJ = 4, REGS = 4;
};
template <>
struct Acc<32> {
  f32x16 v[4][2];
  static constexpr int MI = 4, NJ = 2, REGS = 16;
};

template <int MODE, int SH, bool PRIO>  // MODE 0: store bf16 C; 1: loss against R
__global__ __launch_bounds__(NTH) void k_gemm_bf16_nt(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                      const uint16_t* __restrict__ R, uint16_t* __restrict__ C,
                                                      double* __restrict__ part, int64_t T, int64_t N, int64_t K,
                                                      int64_t ldx, int64_t ldw, int64_t ldr) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  // XCD-aware tile order: the 8 n-tiles of one t-tile are consecutive tile ids on one XCD
  const int nb = gridDim.x, b = blockIdx.x;
  const int per = nb >> 3;
  const int idx = (b & 7) * per + (b >> 3);
  const int ntn = (int)(N / BN);
  const int64_t t0 = (int64_t)(idx / ntn) * BM, n0 = (int64_t)(idx % ntn) * BN;
  const int nk = (int)(K / BK);
  using A_ = Acc<SH>;
  A_ acc;
#pragma unroll
  for (int i = 0; i < A_::MI; ++i)
#pragma unroll
    for (int j = 0; j < A_::NJ; ++j)
#pragma unroll
      for (int r = 0; r < A_::REGS; ++r) acc.v[i][j][r] = 0.f;

  stage_rows(X, ldx, t0, 0, lds, w, lane);
  stage_rows(W, ldw, n0, 0, lds + STAGE_A, w, lane);
  if (nk > 1) {
    stage_rows(X, ldx, t0, BK, lds + STAGE, w, lane);
    stage_rows(W, ldw, n0, BK, lds + STAGE + STAGE_A, w, lane);
  }
  for (int s = 0; s < nk; ++s) {
    if (s + 2 < nk) {
      uint8_t* st = lds + ((s + 2) & (NST - 1)) * STAGE;
      stage_rows(X, ldx, t0, (int64_t)(s + 2) * BK, st, w, lane);
      stage_rows(W, ldw, n0, (int64_t)(s + 2) * BK, st + STAGE_A, w, lane);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (s + 1 < nk) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const uint8_t* st = lds + (s & (NST - 1)) * STAGE;
    if constexpr (SH == 16) {
      bf16x8 a[8], bb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = frag_c(st + STAGE_A, wn * 64 + j * 16 + (lane & 15), lane >> 4);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = frag_c(st, wm * 128 + i * 16 + (lane & 15), lane >> 4);
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc.v[i][j], 0, 0, 0);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        bf16x8 a[4], bb[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) bb[j] = frag_c(st + STAGE_A, wn * 64 + j * 32 + (lane & 31), ks * 2 + (lane >> 5));
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = frag_c(st, wm * 128 + i * 32 + (lane & 31), ks * 2 + (lane >> 5));
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], bb[j], acc.v[i][j], 0, 0, 0);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
      }
    }
  }

  // epilogue.  16x16x32: col = lane & 15, row = (lane >> 4) * 4 + r;
  // 32x32x16: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < A_::MI; ++i)
#pragma unroll
    for (int j = 0; j < A_::NJ; ++j)
#pragma unroll
      for (int r = 0; r < A_::REGS; ++r) {
        int64_t t, n;
        if constexpr (SH == 16) {
          t = t0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
          n = n0 + wn * 64 + j * 16 + (lane & 15);
        } else {
          t = t0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          n = n0 + wn * 64 + j * 32 + (lane & 31);
        }
        if constexpr (MODE == 0) {
          C[t * N + n] = f2bf(acc.v[i][j][r]);
        } else {
          const float o = bf2f(f2bf(acc.v[i][j][r]));
          const float d = bf2f(f2bf(o - bf2f(R[t * ldr + n])));
          sum += d * d;
        }
      }
  if constexpr (MODE == 1) {
    double ds = sum;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ds += __shfl_xor(ds, off);
    double* wsum = reinterpret_cast<double*>(lds);  // the ring is free: one __shared__ object only (guide §5 trap 4a)
    __syncthreads();
    if (lane == 0) wsum[w] = ds;
    __syncthreads();
    if (tid == 0) {
      double tt = 0;
      for (int i = 0; i < 8; ++i) tt += wsum[i];
      part[idx] = tt;
    }
  }
}

// Pipelined variant: 3 steps of glds in flight (issue step s + 3 at iteration s), and the fragments
// of step s + 1 read from LDS (into the other register set) before the MFMAs of step s, so the
// ds_read latency after each barrier hides behind MFMAs instead of idling the matrix pipe.
template <int SH>
struct Frags;
template <>
struct Frags<16> {
  bf16x8 a[8], b[4];
  __device__ __forceinline__ void load(const uint8_t* st, int wm, int wn, int lane) {
#pragma unroll
    for (int j = 0; j < 4; ++j) b[j] = frag_c(st + STAGE_A, wn * 64 + j * 16 + (lane & 15), lane >> 4);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = frag_c(st, wm * 128 + i * 16 + (lane & 15), lane >> 4);
  }
  __device__ __forceinline__ void mma(Acc<16>& acc) const {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc.v[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], b[j], acc.v[i][j], 0, 0, 0);
  }
};
template <>
struct Frags<32> {
  bf16x8 a[2][4], b[2][2];
  __device__ __forceinline__ void load(const uint8_t* st, int wm, int wn, int lane) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int j = 0; j < 2; ++j) b[ks][j] = frag_c(st + STAGE_A, wn * 64 + j * 32 + (lane & 31), ks * 2 + (lane >> 5));
#pragma unroll
      for (int i = 0; i < 4; ++i) a[ks][i] = frag_c(st, wm * 128 + i * 32 + (lane & 31), ks * 2 + (lane >> 5));
    }
  }
  __device__ __forceinline__ void mma(Acc<32>& acc) const {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc.v[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[ks][i], b[ks][j], acc.v[i][j], 0, 0, 0);
  }
};

template <int MODE, int SH>
__global__ __launch_bounds__(NTH) void k_gemm_pipe(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                   const uint16_t* __restrict__ R, uint16_t* __restrict__ C,
                                                   double* __restrict__ part, int64_t T, int64_t N, int64_t K,
                                                   int64_t ldx, int64_t ldw, int64_t ldr) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;
  const int nb = gridDim.x, b = blockIdx.x;
  const int per = nb >> 3;
  const int idx = (b & 7) * per + (b >> 3);
  const int ntn = (int)(N / BN);
  const int64_t t0 = (int64_t)(idx / ntn) * BM, n0 = (int64_t)(idx % ntn) * BN;
  const int nk = (int)(K / BK);  // even, >= 4 (host-checked)
  using A_ = Acc<SH>;
  A_ acc;
#pragma unroll
  for (int i = 0; i < A_::MI; ++i)
#pragma unroll
    for (int j = 0; j < A_::NJ; ++j)
#pragma unroll
      for (int r = 0; r < A_::REGS; ++r) acc.v[i][j][r] = 0.f;
  auto issue = [&](int s) {
    uint8_t* st = lds + (s & (NST - 1)) * STAGE;
    stage_rows(X, ldx, t0, (int64_t)s * BK, st, w, lane);
    stage_rows(W, ldw, n0, (int64_t)s * BK, st + STAGE_A, w, lane);
  };
  issue(0);
  issue(1);
  issue(2);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // step 0 landed (this wave's part)
  __builtin_amdgcn_s_barrier();
  Frags<SH> fa, fb;
  fa.load(lds, wm, wn, lane);
  // iteration s: issue step s + 3, wait for step s + 1, barrier, read step s + 1's fragments, MMA step s
  for (int s = 0; s < nk; s += 2) {
    if (s + 3 < nk) {
      issue(s + 3);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (s + 2 < nk) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every fragment read of an older stage is done (WAR)
    __builtin_amdgcn_s_barrier();
    fb.load(lds + ((s + 1) & (NST - 1)) * STAGE, wm, wn, lane);
    fa.mma(acc);
    // odd half: step s + 1 in fb; read step s + 2 into fa
    if (s + 4 < nk) {
      issue(s + 4);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else if (s + 3 < nk) {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every fragment read of an older stage is done (WAR)
    __builtin_amdgcn_s_barrier();
    if (s + 2 < nk) fa.load(lds + ((s + 2) & (NST - 1)) * STAGE, wm, wn, lane);
    fb.mma(acc);
  }

  float sum = 0.f;
#pragma unroll
  for (int i = 0; i < A_::MI; ++i)
#pragma unroll
    for (int j = 0; j < A_::NJ; ++j)
#pragma unroll
      for (int r = 0; r < A_::REGS; ++r) {
        int64_t t, n;
        if constexpr (SH == 16) {
          t = t0 + wm * 128 + i * 16 + (lane >> 4) * 4 + r;
          n = n0 + wn * 64 + j * 16 + (lane & 15);
        } else {
          t = t0 + wm * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          n = n0 + wn * 64 + j * 32 + (lane & 31);
        }
        if constexpr (MODE == 0) {
          C[t * N + n] = f2bf(acc.v[i][j][r]);
        } else {
          const float o = bf2f(f2bf(acc.v[i][j][r]));
          const float d = bf2f(f2bf(o - bf2f(R[t * ldr + n])));
          sum += d * d;
        }
      }
  if constexpr (MODE == 1) {
    double ds = sum;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) ds += __shfl_xor(ds, off);
    double* wsum = reinterpret_cast<double*>(lds);
    __syncthreads();
    if (lane == 0) wsum[w] = ds;
    __syncthreads();
    if (tid == 0) {
      double tt = 0;
      for (int i = 0; i < 8; ++i) tt += wsum[i];
      part[idx] = tt;
    }
  }
}
}  // namespace

typedef void (*KFn)(const uint16_t*, const uint16_t*, const uint16_t*, uint16_t*, double*, int64_t, int64_t, int64_t,
                    int64_t, int64_t, int64_t);
// mode: bit 0 = loss (else store C); bit 1 = 32x32x16 MFMA; bit 2 = s_setprio around the MFMA block;
// bit 3 = the pipelined variant (bit 2 ignored)
extern "C" int qzp_gemm_nt(const void* X, const void* W, const void* R, void* C, double* part, int64_t T, int64_t N,
                           int64_t K, int64_t ldx, int64_t ldw, int64_t ldr, int mode, void* stream) {
  if (T % BM || N % BN || K % BK || ((T / BM) * (N / BN)) % 8) return -1;
  if ((mode & 8) && ((K / BK) % 2 || K / BK < 4)) return -1;
  static const KFn fns[12] = {k_gemm_bf16_nt<0, 16, false>, k_gemm_bf16_nt<1, 16, false>, k_gemm_bf16_nt<0, 32, false>,
                              k_gemm_bf16_nt<1, 32, false>, k_gemm_bf16_nt<0, 16, true>,  k_gemm_bf16_nt<1, 16, true>,
                              k_gemm_bf16_nt<0, 32, true>,  k_gemm_bf16_nt<1, 32, true>,  k_gemm_pipe<0, 16>,
                              k_gemm_pipe<1, 16>,           k_gemm_pipe<0, 32>,           k_gemm_pipe<1, 32>};
  mode = (mode & 8) ? 8 + (mode & 3) : (mode & 7);
  const unsigned blocks = (unsigned)((T / BM) * (N / BN));
  hipLaunchKernelGGL(fns[mode], dim3(blocks), dim3(NTH), 0, (hipStream_t)stream, (const uint16_t*)X,
                     (const uint16_t*)W, (const uint16_t*)R, (uint16_t*)C, part, T, N, K, ldx, ldw, ldr);
  return (int)hipGetLastError();
}
