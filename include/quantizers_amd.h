/*
 * quantizers_amd.h -- C ABI of the MI355X (gfx950) weight-quantization library.
 *
 * This is the drop-in boundary for the reference's per-linear quantize step.  The reference
 * (mratsim/quantizers) has no native code and no FFI of its own: the step runs inside
 * llmcompressor.oneshot(...) (scripts/do_oneshot.py:179-187) and
 * model.save_pretrained(save_compressed=True) (scripts/do_oneshot.py:197), i.e. in
 * compressed-tensors' calculate_qparams / quantize / fake_quantize / pack_to_int32 /
 * pack_fp4_to_uint8 and llmcompressor's AWQ helpers.  Each entry point below names the
 * reference-side function it replaces; INTEGRATION.md shows the ctypes stub a maintainer would
 * add.  All buffers are DEVICE pointers owned by the caller; nothing here allocates, frees or
 * synchronises.  Every call only enqueues work on `stream` (a hipStream_t, NULL = legacy
 * default stream) and is safe to call from several host threads (one device per thread), with
 * two caller-side conditions: a workspace or sync region is never shared by calls that may run
 * at the same time (the statistics workspace, qz_quantize_nvfp4's sync region: one per stream),
 * and qz_expert_gemms serialises its callers internally (one hipBLASLt handle per device).
 *
 * Weights are bf16 (the dtype do_oneshot.py:88 loads models in), given as a batch of 2-D
 * slices: element (b, r, c) lives at w[b*ld_batch + r*ld_row + c] (elements, not bytes), so
 * both per-expert nn.Linear weights and fused [E, N, K] expert parameters are served
 * (SURVEY.md finding 5).  Outputs are always dense, batch-major.
 *
 * Return value: 0 = success; < 0 = argument error (the cases compressed-tensors raises
 * ValueError for); > 0 = the hipError_t of a failed launch.  qz_strerror() names codes.
 */
#ifndef QUANTIZERS_AMD_H
#define QUANTIZERS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* qz_stream_t; /* hipStream_t */

/* QuantizationArgs.type */
enum { QZ_INT = 0, QZ_FLOAT = 1 };
/* QuantizationArgs.strategy */
enum { QZ_TENSOR = 0, QZ_CHANNEL = 1, QZ_GROUP = 2, QZ_BLOCK = 3, QZ_TENSOR_GROUP = 4 };
/* scale storage: NATIVE = weight dtype (bf16, decision D3); E4M3 = NVFP4 scale_dtype;
 * E8M0 = MXFP4 exponent bytes */
enum { QZ_SCALE_NATIVE = 0, QZ_SCALE_E4M3 = 2, QZ_SCALE_E8M0 = 3 };

/* what qz_quantize writes to q_out (compressed-tensors compression formats) */
enum {
  QZ_OUT_PACKED_INT32 = 0, /* pack-quantized: int32 [rows, cols*bits/32], nibble i of word j = col 8j+i (bits=4) */
  QZ_OUT_INT8 = 1,         /* int-quantized / module weight before packing: int8 [rows, cols] */
  QZ_OUT_FP8 = 2,          /* float-quantized: float8_e4m3fn bytes [rows, cols] */
  QZ_OUT_FP4_PACKED = 3,   /* nvfp4/mxfp4-pack-quantized: uint8 [rows, cols/2], even col in low nibble */
  QZ_OUT_FAKEQUANT = 4     /* fake_quantize: bf16 [rows, cols] = dequantize(quantize(w)) */
};

/* Mirrors the compressed-tensors QuantizationArgs fields the reference's recipes use
 * (configs/recipes/recipe_awq_w4a16.yaml:16-24, recipe_mixed_fp8_int4.yaml:9-24,
 *  recipe_Minimax-M2.1-AWQ-MixedPrec.yaml:24-48, recipe_MoE_RTN_NVFP4.yaml:17-21). */
typedef struct qz_args {
  int32_t num_bits;   /* 2..8 int; 8 (e4m3) or 4 (e2m1) float */
  int32_t type;       /* QZ_INT / QZ_FLOAT */
  int32_t symmetric;  /* 1 / 0 (float requires 1) */
  int32_t strategy;   /* QZ_TENSOR .. QZ_TENSOR_GROUP */
  int32_t group_size; /* GROUP / TENSOR_GROUP */
  int32_t block_h;    /* BLOCK: block_structure[0] */
  int32_t block_w;    /* BLOCK: block_structure[1] */
  int32_t scale_fmt;  /* QZ_SCALE_* */
} qz_args;

/* Error codes */
enum {
  QZ_OK = 0,
  QZ_ERR_NULL = -1,         /* a required pointer is NULL */
  QZ_ERR_SHAPE = -2,        /* negative / zero-sized dims where not allowed */
  QZ_ERR_GROUP = -3,        /* cols % group_size != 0 ("tensor column shape must be divisible by group_size") */
  QZ_ERR_BLOCK = -4,        /* rows/cols not divisible by block ("Block quantization requires exact division") */
  QZ_ERR_BITS = -5,         /* num_bits unsupported for type / output format */
  QZ_ERR_ASYM_FLOAT = -6,   /* "Asymmetric Quantization is not supported for FP4/FP8" */
  QZ_ERR_FORMAT = -7,       /* output format incompatible with args */
  QZ_ERR_WORKSPACE = -8,    /* workspace smaller than qz_quantize_workspace_size() */
  QZ_ERR_ALIGN = -9,        /* pointer/ld alignment violated where required */
  QZ_ERR_UNAVAILABLE = -10  /* a runtime dependency is not loaded / refused the call (qz_expert_gemms: hipBLASLt) */
};

const char* qz_strerror(int code);
int qz_version(void); /* MAJOR*10000 + MINOR*100 + PATCH */
/* Compile-time tuning constants of this build ("key=value;..."; e.g. nt_bytes_q = weight bytes
 * per quantize launch above which the group path streams non-temporally).  Benchmarks and
 * profiles derive the kernel instantiation names they report from it.  No reference
 * counterpart (build metadata). */
const char* qz_build_config(void);

/* Bytes of device workspace qz_quantize / qz_fake_quantize need for these args (0 for the
 * single-pass group path).  The workspace needs no initialisation. */
size_t qz_quantize_workspace_size(int64_t batch, int64_t rows, int64_t cols, const qz_args* a);

/*
 * qz_quantize -- memoryless observe + calculate_qparams + quantize (+ pack), one weight batch.
 * Replaces, per targeted Linear: the memoryless_minmax weight observer -> calculate_qparams
 * ([3P] compressed-tensors, called from llmcompressor during oneshot, do_oneshot.py:179) and
 * the compressor's quantize(..., dtype=int8) -> pack_to_int32 / float8 cast /
 * pack_fp4_to_uint8 (save_pretrained(save_compressed=True), do_oneshot.py:197).
 *   scale_out : bf16 / e4m3 / e8m0 per group; shape [batch][groups] where groups is
 *               rows*cols/g (GROUP, TENSOR_GROUP), rows (CHANNEL), 1 (TENSOR),
 *               (rows/bh)*(cols/bw) (BLOCK)
 *   zp_out    : int8 per group (may be NULL; written as 0 for symmetric)
 *   gscale_out: f32 [batch] NVFP4 global scale (TENSOR_GROUP only; otherwise may be NULL)
 */
int qz_quantize(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row,
                int64_t ld_batch, const qz_args* a, int32_t out_fmt, void* q_out,
                void* scale_out, int8_t* zp_out, float* gscale_out, void* workspace,
                size_t workspace_bytes, qz_stream_t stream);

/*
 * qz_quantize_many -- qz_quantize over n independent weights of one shape and one scheme (e.g.
 * the same projection of every layer), one launch per weight, enqueued in order on `stream`
 * from a single host call.  Replaces the compressor's per-module loop over targeted Linears
 * (save_pretrained(save_compressed=True), do_oneshot.py:197) for callers that hold many
 * same-shape weights; each item is exactly a qz_quantize call.  w / q_out / scale_out are
 * arrays of n device pointers; zp_out / gscale_out may be NULL (no item needs them) or arrays
 * of n pointers.  The workspace is reused by every item (stream order).  Returns the first
 * non-zero status (items before it are enqueued).
 */
int qz_quantize_many(int64_t n, const void* const* w, void* const* q_out, void* const* scale_out,
                     int8_t* const* zp_out, float* const* gscale_out, int64_t batch, int64_t rows,
                     int64_t cols, int64_t ld_row, int64_t ld_batch, const qz_args* a,
                     int32_t out_fmt, void* workspace, size_t workspace_bytes, qz_stream_t stream);

/*
 * qz_quantize_grouped -- qz_quantize over n independent dense [rows, cols] weights of one shape
 * and one scheme in ONE launch (grid.y = weight), like a grouped GEMM: the per-launch ramp-up and
 * drain (~3 us on MI355X) is paid once for the group instead of once per weight.  Replaces the
 * same per-module compressor loop as qz_quantize_many (do_oneshot.py:197).  `table` is a DEVICE
 * array of 4*n uint64 written by the caller before the launch (stream order):
 *   table[i] = weight i (bf16, dense, 16-B aligned), table[n+i] = its codes (16-B aligned: the
 *   kernels store 4- to 16-byte code words), table[2n+i] = its scales (2-B aligned),
 *   table[3n+i] = its int8 zero points (required for asymmetric schemes, else 0).
 * Output layouts are exactly qz_quantize's with batch = 1.  No weight may alias any output.
 * Single-pass group schemes (GROUP / TENSOR_GROUP with a power-of-two group 8..512, int / FP8 /
 * MXFP4 / FP4, not NVFP4 and not fake-quant) and, from round 5, FP8_BLOCK 128 x 128 (e4m3 codes,
 * rows and cols multiples of 128; the strip kernel of qz_block.hip, table[3n+i] unused): anything
 * else returns QZ_ERR_FORMAT and the caller uses qz_quantize_many.  n <= 65535.  No workspace.
 */
int qz_quantize_grouped(int64_t n, const uint64_t* table, int64_t rows, int64_t cols,
                        const qz_args* a, int32_t out_fmt, qz_stream_t stream);

/*
 * qz_quantize_grouped_var -- qz_quantize_grouped over n weights of DIFFERENT shapes and one scheme
 * in ONE launch: every same-scheme linear of a model (Qwen3-4B int4 g128: 252 linears of 5 shapes)
 * pays the launch ramp and drain once (compressor.CompressionPlan).  Same replaced loop as
 * qz_quantize_grouped (do_oneshot.py:197).  `rows`, `cols` are HOST arrays [n], validated as
 * qz_quantize_grouped validates one shape; equal consecutive shapes form a segment and at most 8
 * segments are allowed (sort the weights by shape), else QZ_ERR_SHAPE.  `table` is the DEVICE
 * table of qz_quantize_grouped (4*n uint64: weights, codes, scales, zero points or 0), in the
 * same order.  Outputs exactly qz_quantize's.  n <= 65535.  qz_grouped_blocks(rows, cols) is the
 * number of workgroups one weight takes in such a launch.
 */
int64_t qz_grouped_blocks(int64_t rows, int64_t cols);
int qz_quantize_grouped_var(int64_t n, const uint64_t* table, const int64_t* rows, const int64_t* cols,
                            const qz_args* a, int32_t out_fmt, qz_stream_t stream);

/*
 * qz_quantize_nvfp4 / qz_quantize_grouped_nvfp4 -- NVFP4 (TENSOR_GROUP, FP4 E2M1, group 16, e4m3
 * group scales, f32 per-slice global scale) in TWO launches and no workspace fills.  Replaces the
 * same observer -> calculate_qparams -> quantize -> pack_fp4_to_uint8 chain as qz_quantize
 * (oneshot, scripts/do_oneshot.py:179-187; save_pretrained(save_compressed=True), :197) for the
 * reference's NVFP4 recipes (configs/recipes/recipe_MoE_RTN_NVFP4.yaml:16-21,
 * recipe_Dense_NVFP4.yaml:7-12; scheme preset NVFP4), with results identical to qz_quantize's.
 * The first launch reduces every slice's |w| maximum into `sync`, the second encodes (each slice
 * is read twice: its global scale needs the whole slice first).
 *   qz_quantize_nvfp4: a batch of dense-row slices, slice b at w + b * ld_batch (ld_batch % 8 == 0,
 *     w 16-B aligned); outputs as qz_quantize's (codes uint8 [batch][rows][cols/2], scales e4m3
 *     [batch][rows][cols/16], gscale f32 [batch]).
 *   qz_quantize_grouped_nvfp4: n independent dense [rows, cols] weights of one shape in the same
 *     two launches, DEVICE table of 4*n uint64 {weights, codes, scales, global-scale pointers}
 *     (qz_quantize_grouped's layout with the zero-point row replaced by each weight's f32 global
 *     scale).
 * `sync`: caller-owned DEVICE region of qz_nvfp4_sync_size(slices) bytes, 16-B aligned, ZERO
 * before its first use; every call leaves it zero.  Do not share one region between calls that
 * may run concurrently (e.g. on two streams).
 */
size_t qz_nvfp4_sync_size(int64_t n_slices);
int qz_quantize_nvfp4(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_batch, const qz_args* a,
                      void* q_out, void* scale_out, float* gscale_out, void* sync, size_t sync_bytes,
                      qz_stream_t stream);
int qz_quantize_grouped_nvfp4(int64_t n, const uint64_t* table, int64_t rows, int64_t cols, const qz_args* a,
                              void* sync, size_t sync_bytes, qz_stream_t stream);

/*
 * qz_quantize_qparams -- quantize with caller-supplied qparams (stateful observers such as the
 * recipes' `minmax`, recipe_Minimax-M2.1-AWQ-MixedPrec.yaml:48).  Replaces [3P]
 * compressed-tensors quantize(x, scale, zero_point, args) / fake_quantize(...).
 * scale/zp/gscale have the qz_quantize output layouts; zp may be NULL for symmetric.
 */
int qz_quantize_qparams(const void* w, int64_t batch, int64_t rows, int64_t cols,
                        int64_t ld_row, int64_t ld_batch, const qz_args* a, int32_t out_fmt,
                        const void* scale, const int8_t* zp, const float* gscale, void* q_out,
                        qz_stream_t stream);

/*
 * qz_observe_minmax -- per-group amin/amax of the weight in bf16 (exact), the observation
 * step of [3P] llmcompressor's observers (flatten_for_calibration + amin/amax).  Outputs
 * are bf16 [batch][groups] (TENSOR_GROUP -> GROUP layout).
 */
int qz_observe_minmax(const void* w, int64_t batch, int64_t rows, int64_t cols,
                      int64_t ld_row, int64_t ld_batch, const qz_args* a, void* min_out,
                      void* max_out, void* workspace, size_t workspace_bytes,
                      qz_stream_t stream);

/*
 * qz_calculate_qparams -- [3P] compressed-tensors calculate_qparams(min, max, args,
 * global_scale) over n groups given bf16 min/max.  gscale (f32, may be NULL) is one value
 * for all n groups.
 */
int qz_calculate_qparams(const void* min_vals, const void* max_vals, int64_t n,
                         const qz_args* a, const float* gscale, void* scale_out,
                         int8_t* zp_out, qz_stream_t stream);

/*
 * qz_dequantize -- [3P] compressed-tensors dequantize / the decompressors: codes in the
 * qz_quantize q_out layout (PACKED_INT32, INT8, FP8, FP4_PACKED) -> bf16 [batch][rows][cols].
 */
int qz_dequantize(const void* q, int64_t batch, int64_t rows, int64_t cols, const qz_args* a,
                  int32_t in_fmt, const void* scale, const int8_t* zp, const float* gscale,
                  void* w_out, qz_stream_t stream);

/*
 * qz_pack_int32 -- [3P] compressed-tensors pack_to_int32(value, num_bits, packed_dim):
 * int8 [rows, cols] -> int32 [rows, ceil(cols*bits/32)] (packed_dim 1) or
 * [ceil(rows*bits/32), cols] (packed_dim 0, the asymmetric weight_zero_point layout).
 */
int qz_pack_int32(const int8_t* v, int64_t rows, int64_t cols, int32_t num_bits,
                  int32_t packed_dim, int32_t* out, qz_stream_t stream);

/* ---------------------------------------------------------------- AWQ */

/*
 * qz_awq_absmean_accum -- adds sum_t |x[t, c]| (fp32, decision D8) into sum[c] for a bf16
 * activation block x [tokens, channels] (row stride ld).  Replaces the running mean|x| of
 * [3P] llmcompressor AWQModifier's cache_smooth_activations_hook (_accumulate_mean).
 * Deterministic: fixed-order reduction through `workspace` (qz_awq_absmean_workspace_size
 * bytes), in ONE launch: the last-arriving workgroup of each column window sums the window's
 * row-chunk partials.  Statistics workspace contract (absmean and w_mean): its first
 * QZ_STATS_HEAD_BYTES bytes are arrival counters that must be zero before the first call on that
 * workspace (e.g. one hipMemset when it is allocated); every call leaves them zero again.  Do
 * not share a statistics workspace with other entry points or between concurrent streams.
 */
#define QZ_STATS_HEAD_BYTES 32768
size_t qz_awq_absmean_workspace_size(int64_t tokens, int64_t channels);
int qz_awq_absmean_accum(const void* x, int64_t tokens, int64_t channels, int64_t ld,
                         float* sum, void* workspace, size_t workspace_bytes,
                         qz_stream_t stream);

/*
 * qz_awq_weight_mean_accum -- adds sum_r |W[r,c]| / (absmax(group(r,c)) + 1e-6) (bf16
 * elementwise, fp64 sum) into wsum[c] for one balance layer W [rows, cols].  group_size =
 * the layer's quantization group (cols for channel strategy).  Replaces [3P] llmcompressor
 * _compute_layer_means.  Deterministic: fixed-order reduction through `workspace`
 * (qz_awq_weight_mean_workspace_size bytes, 8-B aligned; may be 0 bytes for the generic path),
 * one launch for power-of-two groups of 8..512 (the statistics workspace contract above).
 */
size_t qz_awq_weight_mean_workspace_size(int64_t rows, int64_t cols, int32_t group_size);
int qz_awq_weight_mean_accum(const void* w, int64_t rows, int64_t cols, int64_t ld,
                             int32_t group_size, double* wsum, void* workspace,
                             size_t workspace_bytes, qz_stream_t stream);

/*
 * Segmented statistics (round 5) -- n <= 16 independent operands of one column count in ONE
 * launch: segment s adds exactly what its own single call would (qz_awq_absmean_accum(x[s],
 * tokens[s], channels, ld[s], sums[s], ...) / qz_awq_weight_mean_accum(w[s], rows[s], cols,
 * ld[s], group_size, wsums[s], ...)), bit for bit: the same chunking and reduction tree per
 * segment.  The output pointers must be distinct.  Returns QZ_ERR_FORMAT, launching nothing, when
 * a segment would not take the single call's one-launch plan (unaligned or wide-ld operands,
 * too many counters; the *_workspace_size functions then return 0): issue single calls instead.
 * Replaces the per-sample calls of the AWQ activation hook over one batched calibration forward
 * and the per-balance-layer calls of _compute_layer_means for one mapping.  The statistics
 * workspace contract above applies.
 */
size_t qz_awq_absmean_segments_workspace_size(int32_t n, const int64_t* tokens, int64_t channels);
int qz_awq_absmean_accum_segments(int32_t n, const void* const* x, const int64_t* tokens,
                                  int64_t channels, const int64_t* ld, float* const* sums,
                                  void* workspace, size_t workspace_bytes, qz_stream_t stream);
size_t qz_awq_weight_mean_segments_workspace_size(int32_t n, const int64_t* rows, int64_t cols,
                                                  int32_t group_size);
int qz_awq_weight_mean_accum_segments(int32_t n, const void* const* w, const int64_t* rows,
                                      int64_t cols, const int64_t* ld, int32_t group_size,
                                      double* const* wsums, void* workspace,
                                      size_t workspace_bytes, qz_stream_t stream);

/*
 * qz_awq_stats_layout -- the reduction plan the statistics calls use for a [rows, cols] input
 * (which = 0: absmean, rows = tokens; 1: w_mean with group_size): out[0] one-launch (1) or
 * two-launch (0), out[1] column window, out[2] rows per chunk, out[3] chunks, out[4] row slots
 * per workgroup, out[5] final-sum thread groups, out[6] counter head bytes.  Lets a caller (or a
 * test) restate the fixed summation order exactly.  No reference counterpart.
 */
int qz_awq_stats_layout(int32_t which, int64_t rows, int64_t cols, int32_t group_size, int64_t* out);

/*
 * qz_awq_sq_err_accum -- the grid search's loss numerator: *out += sum over [rows, cols] of
 * f32(bf16(a - b))^2 for two bf16 parent outputs (reference output and the output with the
 * fake-quantized balance layers), summed in f64 in a fixed order (deterministic).  Replaces
 * the `(fp16_out - q_out).pow(2).sum()` of [3P] llmcompressor AWQModifier._compute_loss.
 * workspace: qz_awq_sq_err_workspace_size(rows, cols) bytes.
 */
size_t qz_awq_sq_err_workspace_size(int64_t rows, int64_t cols);
int qz_awq_sq_err_accum(const void* a, const void* b, int64_t rows, int64_t cols, int64_t lda,
                        int64_t ldb, double* out, void* workspace, size_t workspace_bytes,
                        qz_stream_t stream);

/*
 * The same loss in two phases, for a search that evaluates many (grid point, expert) losses
 * before it needs any of them: qz_awq_sq_err_partials writes the per-block f64 partial sums of
 * one loss into part[0 .. qz_awq_sq_err_partials_count(rows, cols)) (stage 1 of
 * qz_awq_sq_err_accum), and qz_awq_sq_err_reduce then adds n losses' partial rows (row i at
 * part + i * part_ld) into out[i] with stage 2's fixed order -- one launch for the whole search;
 * out[i] is bit-identical to qz_awq_sq_err_accum on the same outputs.
 */
int64_t qz_awq_sq_err_partials_count(int64_t rows, int64_t cols);
int qz_awq_sq_err_partials(const void* a, const void* b, int64_t rows, int64_t cols, int64_t lda,
                           int64_t ldb, double* part, qz_stream_t stream);
int qz_awq_sq_err_reduce(const double* part, int64_t n, int64_t nb, int64_t part_ld, double* out,
                         qz_stream_t stream);
/*
 * qz_awq_sq_err_partials_multi -- qz_awq_sq_err_partials for 1..8 outputs b[0..n_b) (a HOST array
 * of device pointers) against one reference a, all dense [rows, cols] bf16 (cols % 8 == 0,
 * 16-B aligned): output g's partials go to part + g * part_ld, bit-identical to a
 * qz_awq_sq_err_partials(a, b[g]) call, while a is read once for all of them.
 */
int qz_awq_sq_err_partials_multi(const void* a, const void* const* b, int32_t n_b, int64_t rows,
                                 int64_t cols, double* part, int64_t part_ld, qz_stream_t stream);

/*
 * qz_awq_grid_scales -- one grid point of [3P] AWQModifier._compute_best_scale (fp32):
 * s = clamp(x_mean^r / (w_mean^(1-r) + 1e-4), 1e-4) (duo) or clamp(x_mean^r, 1e-4);
 * s /= sqrt(max(s) * min(s)); inf/nan -> 1.  Single workgroup; channels <= 65536.
 */
int qz_awq_grid_scales(const float* x_mean, const float* w_mean, int64_t channels,
                       float ratio, int32_t duo_scaling, float* scales_out,
                       qz_stream_t stream);

/*
 * qz_awq_grid_scales_batched -- the same grid point for `batch` independent mappings at once
 * (x_mean / w_mean / scales_out are [batch, channels], row-major): every MoE expert's
 * w3 -> w2 (up_proj -> down_proj) mapping of one layer in one launch.  Results are identical
 * to `batch` calls of qz_awq_grid_scales.
 */
int qz_awq_grid_scales_batched(const float* x_mean, const float* w_mean, int64_t batch,
                               int64_t channels, float ratio, int32_t duo_scaling,
                               float* scales_out, qz_stream_t stream);

/*
 * qz_awq_fake_quant -- the grid search's per-balance-layer step W' = Q(W * s) / s with the
 * layer's own scheme, fused into one pass (bf16 products, bf16 fake-quant, f32 column
 * scales).  col_scales may be NULL (plain fake_quantize).  w_out may alias w.
 */
int qz_awq_fake_quant(const void* w, int64_t batch, int64_t rows, int64_t cols, int64_t ld_row,
                      int64_t ld_batch, const qz_args* a, const float* col_scales, void* w_out,
                      void* workspace, size_t workspace_bytes, qz_stream_t stream);

/*
 * qz_awq_fake_quant_batched -- qz_awq_fake_quant over a batch of slices with one column-scale
 * vector per slice: col_scales[b * cs_ld_batch + c] (cs_ld_batch >= cols; 0 = shared).  The
 * batched grid step of per-expert AWQ mappings (each expert's w2 with its own scales).
 */
int qz_awq_fake_quant_batched(const void* w, int64_t batch, int64_t rows, int64_t cols,
                              int64_t ld_row, int64_t ld_batch, const qz_args* a,
                              const float* col_scales, int64_t cs_ld_batch, void* w_out,
                              void* workspace, size_t workspace_bytes, qz_stream_t stream);

/*
 * qz_scale_columns / qz_scale_rows -- AWQ _apply_smoothing: in place, bf16-rounded,
 * W[:, c] *= s[c] (balance layers) or W[r, :] /= s[r] (smooth Linear's last rows; a 1-D norm
 * weight is rows=n, cols=1).  divide=1 divides, 0 multiplies.
 */
int qz_scale_columns(void* w, int64_t rows, int64_t cols, int64_t ld, const float* s,
                     int32_t divide, qz_stream_t stream);
int qz_scale_rows(void* w, int64_t rows, int64_t cols, int64_t ld, const float* s,
                  int32_t divide, qz_stream_t stream);

/*
 * qz_moe_combine -- the tail of a fused-experts MoE forward in the eager arithmetic: for every
 * token t, out[t, :] = (((+0 + v_0) + v_1) + ... + v_{k-1}) with a bf16 rounding after each
 * add, where v_j = bf16(expert_out[r, :] * weights[perm[r]]) and r = src[t * top_k + j] is the
 * expert-sorted row of t's j-th expert in ascending expert id.  expert_out is [rows, hidden]
 * bf16 (rows = tokens * top_k), weights the flat routing weights [tokens * top_k] (bf16, or f32
 * when weights_f32), perm / src int64 device arrays, out [tokens, hidden] bf16.  Replaces the
 * per-expert `current * top_k_weights[...]` and bf16 `index_add_` of transformers' eager
 * experts loop (transformers 4.57 modeling_qwen3_moe Qwen3MoeSparseMoeBlock.forward, as pinned
 * by the reference's requirements) -- bit-identical to that loop.
 */
int qz_moe_combine(const void* expert_out, int64_t rows, int64_t hidden, const void* weights,
                   int32_t weights_f32, const int64_t* perm, const int64_t* src, int64_t tokens,
                   int32_t top_k, void* out, qz_stream_t stream);

/*
 * qz_moe_silu_mul -- out[r, c] = bf16(bf16(silu(gate_up[r, c])) * gate_up[r, inter + c]) for the
 * [rows, 2 * inter] bf16 gate/up GEMM output (row stride ld >= 2 * inter) into a dense
 * [rows, inter] bf16 out, with torch's silu arithmetic (x / (1 + exp(-x)) in f32).  Replaces
 * `self.act_fn(gate) * up` of the eager experts loop (transformers 4.57
 * modeling_qwen3_moe.Qwen3MoeMLP / the fused experts' forward); callers verify it against the
 * composed ops on first use (the exp implementation is the device library's).
 */
int qz_moe_silu_mul(const void* gate_up, int64_t rows, int64_t inter, int64_t ld, void* out,
                    qz_stream_t stream);
/*
 * qz_silu_mul -- the same for separate gate and up projections (a dense MLP, e.g. transformers
 * 4.57 modeling_qwen3.Qwen3MLP.forward's `self.act_fn(self.gate_proj(x)) * self.up_proj(x)`):
 * out[r, c] = bf16(bf16(silu(gate[r, c])) * up[r, c]), gate / up bf16 [rows, inter] with row
 * strides ld_gate / ld_up, out dense [rows, inter] bf16.
 */
int qz_silu_mul(const void* gate, int64_t ld_gate, const void* up, int64_t ld_up, int64_t rows, int64_t inter,
                void* out, qz_stream_t stream);

/*
 * qz_expert_gemms -- the per-expert GEMMs of a fixed-routing MoE forward, issued in one call:
 * for i < count, out[row0[i]:row1[i], :n] = x[row0[i]:row1[i], :k] @ w[expert[i]]^T, where
 * w[e] is the [n, k] bf16 matrix at w + e * w_stride (row stride ldw), x / out bf16 with row
 * strides ldx / ldo, all on `stream`.  Each GEMM is the hipBLASLt problem torch.mm(x[rows],
 * w[e].t()) poses (f32 compute; the heuristic's first algorithm under a workspace limit of
 * workspace_bytes), through the hipBLASLt already loaded in the process (PyTorch's); callers
 * verify the bits against torch.mm before relying on them.  Replaces the eager experts loop's
 * per-expert `nn.functional.linear` calls (transformers 4.57 per-expert MLPs, D15) in the
 * fixed-routing forwards of an AWQ grid.  QZ_ERR_UNAVAILABLE without hipBLASLt.
 */
/* qz_expert_gemms_library -- bind qz_expert_gemms to the hipBLASLt at `path`, which must already be
 * loaded in the process (e.g. PyTorch's torch/lib/libhipblaslt.so); nothing is loaded here.  Once
 * per process (the same object again returns 0; another one QZ_ERR_FORMAT).  Without this call
 * the first qz_expert_gemms binds the loaded object with ROCm's soname "libhipblaslt.so.1".
 * qz_expert_gemms_status -- why the last binding / GEMM call was refused ("bound: <path>" when
 * bound).  Thread safety: qz_expert_gemms serialises its callers on one internal mutex (one
 * hipBLASLt handle per device); several host threads on several streams are safe. */
int qz_expert_gemms_library(const char* path);
const char* qz_expert_gemms_status(void);
int qz_expert_gemms(const void* x, int64_t ldx, const void* w, int64_t w_stride, int64_t ldw, int64_t n,
                    int64_t k, void* out, int64_t ldo, const int64_t* row0, const int64_t* row1,
                    const int32_t* expert, int32_t count, void* workspace, size_t workspace_bytes,
                    qz_stream_t stream);

/*
 * qz_rmsnorm128 -- RMSNorm over rows of 128 bf16 (row stride ld, ld % 4 == 0, 8-B aligned) into a
 * dense [rows, 128] bf16 out, in the model's own arithmetic: f32 squares summed in the order of
 * PyTorch's reduce kernel for a 128-wide row (32 threads x 4, shuffle tree), times 1/128, + eps,
 * correctly rounded rsqrt, bf16(x * r), bf16(weight * y) -- bit-identical to transformers 4.57
 * modeling_qwen3.Qwen3RMSNorm.forward for the q / k head norms (head_dim 128)
 * (profiles/r03t_rmsnorm_probe.log); callers still check it on first use.
 */
int qz_rmsnorm128(const void* x, int64_t rows, int64_t ld, const void* weight, float eps, void* out,
                  qz_stream_t stream);

/*
 * qz_rotary128 -- rotary position embedding of 128-wide heads in the model's own arithmetic:
 * out = bf16(bf16(x * cos) + bf16(rotate_half(x) * sin)), rotate_half(x) = cat(-x[64:], x[:64]).
 * x / out: bf16 [B, H, T, 128] with element strides (xb, xh, xt) / (ob, oh, ot), the last dim
 * contiguous; cos / sin: bf16 [B, T, 128] with strides (cb, ct), broadcast over H.  All strides
 * multiples of 4, pointers 8-B aligned.  Replaces transformers 4.57
 * modeling_qwen3.apply_rotary_pos_emb (its three elementwise kernels and the rotate_half cat).
 */
int qz_rotary128(const void* x, int64_t B, int64_t H, int64_t T, int64_t xb, int64_t xh, int64_t xt,
                 const void* cos, const void* sin, int64_t cb, int64_t ct, void* out, int64_t ob, int64_t oh,
                 int64_t ot, qz_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* QUANTIZERS_AMD_H */
