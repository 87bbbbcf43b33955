// qz_block.hip -- FP8_BLOCK (128 x 128 blocks, e4m3 codes, one bf16 scale per block), gfx950.
//
// compressed-tensors' FP8_BLOCK preset: the attention half of the reference's mixed recipe
// (configs/recipes/recipe_mixed_fp8_int4.yaml:9-11, corrected form
// scripts/quantization_multiple_modifiers.py:58-64) and the scheme of its only data-free driver
// (scripts/quant_GLM-4.7-Flash-FP8.py:11-24).  Observer memoryless_minmax over each 128 x 128
// block -> s = bf16(absmax / 448) -> e4m3(clamp(bf16(w / s), +-448)).
//
// One pass, one HBM read.  A workgroup of 256*NB threads covers a 128-row x (128*NB)-column
// strip: NB horizontally adjacent blocks of one block row, held in registers (8 units of 8 bf16
// per thread).  Thread t owns column unit t % (16*NB) of rows t / (16*NB) + 16*i, i < 8, so one
// wave-load reads (4/NB) rows x NB*256 contiguous bytes (the default NB = 2: 512-B row pieces;
// the round-1 tile kernel, k_tile_fast with one block per workgroup, read 256-B pieces).  Block
// |max| on the raw bf16 words (v_pk_max_u16), DPP within the 16 lanes of a block row, lane
// shuffles across the rows a wave holds, then across the 4*NB waves through LDS.  The e4m3 codes of two lanes holding adjacent units of one row are
// exchanged by one DPP swap so every lane writes 16 B (even lanes the even rows of a pair, odd
// lanes the odd rows): 16-B stores instead of 8-B ones.  Everything is shifts: no divisions but the
// workgroup's block coordinates (scalar).
#include <hip/hip_runtime.h>

#include "qz_device.h"

using namespace qz;

// widest strip (blocks per workgroup); the host takes the widest that divides cols / 128.  r05a/b:
// the mixed plan's attention half (q, k+v, o table launches) 464 / 465 / 483 us at NB = 2 / 4 / 1
// (profiles/r05a_tune_block.log, r05b_tune_block.log); per launch the best NB varies by +-3 %.
// Weight loads are non-temporal (default-policy loads 4-8 % slower at every shape, r05a)
#ifndef QZ_BLK_NB
#define QZ_BLK_NB 2
#endif
// Code stores: non-temporal, throughout.  In isolation (scripts/tune_block.py, the same launch back
// to back) write-through (sc1) stores won on the smaller launches -- sc1 / nt = 83.5 / 95.1 us for
// the 566 MB k+v table launch, 45.3 / 49.2 us for a 283 MB batch, but 192.5 / 189.7 (q) and
// 183.6 / 178.4 us (o) for the 1.13 GB launches (r05b); plain stores 85.3 / 197.5 / 192.8 us.  In
// the mixed recipe's whole-model plan (scripts/tune_plan.py RECIPE=mixed, r05f) write-through
// stores for every launch below 768 MiB made the step 2.2 % slower (1512 vs 1479 us) and a 32 MiB
// write-through tail (qz_device.h wt_tail) changed nothing (1482 us), so neither is built.

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct BlkArgs {
  const uint16_t* w;   // batch mode: slice b at w + b * ld_batch
  int64_t ld_batch;    // elements
  int64_t ld_row;      // elements between rows of a slice
  int64_t q_ld_batch;  // batch mode: code bytes per slice (rows * cols)
  uint8_t* q_out;      // batch mode: e4m3 [batch][rows][cols]
  uint16_t* s_out;     // batch mode: bf16 [batch][rows/128][cols/128]
  const uint64_t* tab; // grouped mode: [4][n_tab] {weight, codes, scales, 0}
  int64_t n_tab;
  uint32_t cols;       // codes row length (bytes)
  uint32_t strips_c;   // strips per block row = cols / (128 * NB)
  uint32_t blocks_c;   // scale row length = cols / 128
  uint32_t n_blocks;   // scales per slice
  QP p;
};

__device__ __forceinline__ f32x2 bfr2(f32x2 v) {  // both lanes rounded to bf16 (RNE), widened back
  f32x2 r;
  r.x = __uint_as_float(__builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){0.0f, v.x}, bf16x2)));
  r.y = __uint_as_float(__builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){0.0f, v.y}, bf16x2)));
  return r;
}

// e4m3 codes of one unit (8 bf16 in four words) under the block's qparams: bf16(x / s) (x * rcp(s)
// by the rcp lemma when g.fast), clamp +-448, v_cvt_pk_fp8_f32 (OCP e4m3fn, RNE) --
// encode_store<K_FP8>'s arithmetic (qz_quant.hip)
__device__ __forceinline__ uint2 fp8_unit(const uint4 v, const GP& g) {
  const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
  uint32_t pk[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 x = {__uint_as_float(wd[k] << 16), __uint_as_float(wd[k] & 0xffff0000u)};
    f32x2 t = g.fast ? x * (f32x2){g.rs, g.rs} : (f32x2){x.x / g.s, x.y / g.s};
    t = bfr2(t);
    pk[k] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(__builtin_amdgcn_fmed3f(t.x, -448.f, 448.f),
                                                      __builtin_amdgcn_fmed3f(t.y, -448.f, 448.f), 0, false) & 0xffffu;
  }
  return make_uint2(pk[0] | (pk[1] << 16), pk[2] | (pk[3] << 16));
}

__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {  // lane l <- lane l ^ 1 (DPP quad_perm [1,0,3,2])
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}

template <int NB, bool TAB>
__global__ __launch_bounds__(256 * NB) void k_block_fp8(BlkArgs A) {
  constexpr int UPR = 16 * NB;        // units per strip row
  constexpr int RPI = 256 * NB / UPR;  // rows per load round (16)
  constexpr int IT = 128 / RPI;        // units per thread (8)
  __shared__ __attribute__((aligned(16))) uint32_t red[NB][4 * NB];  // per block, per wave |max|
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const uint32_t s = blockIdx.x;
  const uint32_t br = s / A.strips_c, bc = s - br * A.strips_c;  // block row, strip (uniform)
  const uint16_t* w;
  uint8_t* q;
  uint16_t* sc;
  if constexpr (TAB) {
    w = reinterpret_cast<const uint16_t*>(A.tab[blockIdx.y]);
    q = reinterpret_cast<uint8_t*>(A.tab[A.n_tab + blockIdx.y]);
    sc = reinterpret_cast<uint16_t*>(A.tab[2 * A.n_tab + blockIdx.y]);
  } else {
    w = A.w + (int64_t)blockIdx.y * A.ld_batch;
    q = A.q_out + (int64_t)blockIdx.y * A.q_ld_batch;
    sc = A.s_out + (int64_t)blockIdx.y * A.n_blocks;
  }
  const uint32_t cu = t & (UPR - 1), rr = t / UPR;
  const int64_t row0 = (int64_t)br * 128, col0 = (int64_t)bc * (128 * NB);
  const uint16_t* src = w + row0 * A.ld_row + col0;  // uniform strip base
  uint4 v[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const u32x4* p = reinterpret_cast<const u32x4*>(src + (uint32_t)((rr + RPI * i) * (uint32_t)A.ld_row + cu * 8));
    const u32x4 x = __builtin_nontemporal_load(p);
    v[i] = make_uint4(x.x, x.y, x.z, x.w);
  }
  // block |max| on the bf16 bit patterns (two per dword)
  uint32_t m = 0;
#pragma unroll
  for (int i = 0; i < IT; ++i)
    m = pk_max_u16(m, pk_max_u16(pk_max_u16(v[i].x & 0x7fff7fffu, v[i].y & 0x7fff7fffu),
                                 pk_max_u16(v[i].z & 0x7fff7fffu, v[i].w & 0x7fff7fffu)));
  uint32_t am = max(m & 0xffffu, m >> 16);
  am = grp_max_u<16>(am);                                  // the 16 lanes of one block row
  if (NB == 1) am = max(am, (uint32_t)__shfl_xor((int)am, 16, 64));
  if (NB <= 2) am = max(am, (uint32_t)__shfl_xor((int)am, 32, 64));
  const int blk = (lane >> 4) & (NB - 1);
  if (lane < UPR && (lane & 15) == 0) red[blk][wv] = am;
  __syncthreads();
  am = 0;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const uint4 r = reinterpret_cast<const uint4*>(&red[blk][0])[k];
    am = max(am, max(max(r.x, r.y), max(r.z, r.w)));
  }
  QP p = A.p;
  p.kind = K_FP8;
  p.sym = 1;
  const GP g = group_params_sym(p, __uint_as_float(am << 16));
  // codes: lanes l, l ^ 1 hold adjacent units of one row; after one swap of 8 B the even lane
  // writes row i (its unit + the odd lane's), the odd lane row i + RPI (the even lane's + its own)
  const bool odd = lane & 1;
  uint8_t* dst = q + row0 * (int64_t)A.cols + col0;
#pragma unroll
  for (int j = 0; j < IT / 2; ++j) {
    const uint2 c0 = fp8_unit(v[2 * j], g), c1 = fp8_unit(v[2 * j + 1], g);
    const uint2 snd = odd ? c0 : c1;
    const uint2 rcv = make_uint2(swap_pair(snd.x), swap_pair(snd.y));
    const uint4 o = odd ? make_uint4(rcv.x, rcv.y, c1.x, c1.y) : make_uint4(c0.x, c0.y, rcv.x, rcv.y);
    const uint32_t row = rr + RPI * (2 * j + (odd ? 1 : 0));
    uint4* d = reinterpret_cast<uint4*>(dst + (uint32_t)(row * A.cols + (cu & ~1u) * 8));
    __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), reinterpret_cast<u32x4*>(d));
  }
  if (t < UPR && (t & 15) == 0) sc[br * A.blocks_c + bc * NB + blk] = (uint16_t)g.sbits;
}

inline bool aligned(const void* p, size_t n) { return ((uintptr_t)p % n) == 0; }

}  // namespace

namespace qz {

// the FP8_BLOCK fast path applies: e4m3, 128 x 128 blocks, dense 16-B aligned rows
bool block_fp8_ok(const BlockFp8Job& J) {
  if (J.rows <= 0 || J.cols <= 0 || J.rows % 128 || J.cols % 128 || J.n <= 0 || J.n > 65535) return false;
  if (J.ld_row < J.cols || J.ld_row % 8 || J.ld_row > (1 << 22)) return false;  // 32-bit offsets in a strip
  if (J.cols > (1 << 24) || (J.rows / 128) * (J.cols / 128) > INT32_MAX) return false;  // grid.x, scale index
  if (J.tab) return aligned(J.tab, 8);
  if (!aligned(J.w, 16) || !aligned(J.q_out, 16) || !aligned(J.s_out, 2)) return false;
  return J.n == 1 || J.ld_batch % 8 == 0;
}

int block_fp8_launch(const BlockFp8Job& J, const QP& p, hipStream_t st) {
  if (!block_fp8_ok(J)) return QZ_ERR_FORMAT;
  const int64_t bc = J.cols / 128;
  const int nb = (QZ_BLK_NB >= 4 && bc % 4 == 0) ? 4 : (QZ_BLK_NB >= 2 && bc % 2 == 0) ? 2 : 1;
  BlkArgs A;
  A.w = (const uint16_t*)J.w;
  A.ld_batch = J.ld_batch;
  A.ld_row = J.ld_row;
  A.q_ld_batch = J.rows * J.cols;
  A.q_out = (uint8_t*)J.q_out;
  A.s_out = (uint16_t*)J.s_out;
  A.tab = J.tab;
  A.n_tab = J.tab ? J.n : 0;
  A.cols = (uint32_t)J.cols;
  A.strips_c = (uint32_t)(bc / nb);
  A.blocks_c = (uint32_t)bc;
  A.n_blocks = (uint32_t)((J.rows / 128) * bc);
  A.p = p;
  const dim3 grid((unsigned)((J.rows / 128) * (bc / nb)), (unsigned)J.n);
  const bool tab = J.tab != nullptr;
  if (nb == 4) {
    if (tab) hipLaunchKernelGGL((k_block_fp8<4, true>), grid, dim3(1024), 0, st, A);
    else hipLaunchKernelGGL((k_block_fp8<4, false>), grid, dim3(1024), 0, st, A);
  } else if (nb == 2) {
    if (tab) hipLaunchKernelGGL((k_block_fp8<2, true>), grid, dim3(512), 0, st, A);
    else hipLaunchKernelGGL((k_block_fp8<2, false>), grid, dim3(512), 0, st, A);
  } else {
    if (tab) hipLaunchKernelGGL((k_block_fp8<1, true>), grid, dim3(256), 0, st, A);
    else hipLaunchKernelGGL((k_block_fp8<1, false>), grid, dim3(256), 0, st, A);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? QZ_OK : (int)e;
}

}  // namespace qz
