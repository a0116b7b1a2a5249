/*! @file gpu.h
 *  @brief Device-pointer, batched and stream-ordered API (no reference
 *  counterpart).
 *
 *  Every vs_* compute function takes device pointers and a stream (a
 *  hipStream_t passed as void*; NULL is the HIP null stream) and is
 *  asynchronous with respect to the host: it only enqueues work.  Temporary
 *  device memory comes from the library's caching pool (blocks tagged with the
 *  stream that used them and an event), so the calls are safe to use from
 *  several streams; after a warm-up call has populated the pool and the plans
 *  (FFT twiddles), steady-state calls allocate nothing.
 *
 *  This is the layer the PyTorch custom ops (veles.simd_amd.ops) and the
 *  multi-GPU layer (veles.simd_amd.parallel) call; the source-compatible C
 *  API in the other headers is built on it.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_GPU_H_
#define VELES_SIMD_GPU_H_

#include <stddef.h>
#include <stdint.h>
#include <simd/common.h>

SIMD_API_BEGIN

typedef void *vs_stream_t;

typedef enum {
  VS_OK = 0,
  VS_ERR_INVALID = 1,      ///< bad argument (message in vs_last_error())
  VS_ERR_HIP = 2,          ///< HIP runtime error
  VS_ERR_NO_GPU = 3,       ///< no usable gfx950 device
  VS_ERR_UNSUPPORTED = 4,  ///< shape/parameter outside what is implemented
  VS_ERR_ALLOC = 5,        ///< allocation failure
  VS_ERR_COMM = 6,         ///< RCCL error (communicator aborted)
  VS_ERR_TIMEOUT = 7       ///< distributed wait exceeded its timeout
} vs_status;

typedef enum {
  VS_F32 = 0,
  VS_F16 = 1,  ///< IEEE binary16 stored as uint16
  VS_I16 = 2,
  VS_I32 = 3,
  VS_U8 = 4
} vs_dtype;

/* ---------------------------------------------------------------- runtime */
const char *vs_version(void);
/// 1 if at least one HIP device is usable (VELES_DISABLE_GPU=1 forces 0).
int vs_gpu_available(void);
int vs_device_count(void);
int vs_set_device(int device);
int vs_get_device(void);
/// Message of the last failing call on this thread ("" if none).
const char *vs_last_error(void);
int vs_is_device_pointer(const void *ptr);
/// Pinned host memory for operands of the reference-compatible host API
/// (<simd/matrix.h>, <simd/convolve.h>, ...).  Calls on pageable arrays
/// copy every operand through the runtime's pinned staging image with the
/// CPU (a 1 MiB memcpy costs more than its PCIe transfer); arrays
/// from vs_host_alloc are recognised by the runtime: read-once inputs and
/// outputs are accessed in place through the GPU mapping, re-read inputs
/// move by asynchronous DMA (matrix_multiply 300 x 256 x 1000: 114-127 us on
/// pageable arrays, 82 us on pinned ones, of which the two PCIe transfers
/// are the larger part).  Pinned tensors of other allocators (hipHostMalloc,
/// torch pin_memory) are treated the same way.  Free with vs_host_free, not
/// free().  Pinning an array the caller already owns (hipHostRegister) is
/// not offered: where the driver cannot pin user pages the attempt leaves
/// the HIP runtime unable to copy from that range afterwards.
void *vs_host_alloc(size_t bytes);
void vs_host_free(void *ptr);
vs_status vs_stream_synchronize(vs_stream_t stream);
/// Number of the architecture the kernels were compiled for (950).
int vs_compiled_arch(void);
/// Returns the library's cached scratch memory to the device.
void vs_release_cached_memory(void);

/* ----------------------------------------------------------- elementwise */
typedef enum { VS_OP_ADD = 0, VS_OP_SUB = 1, VS_OP_MUL = 2 } vs_binary_op;
typedef enum {
  VS_FN_SIN = 0,
  VS_FN_COS = 1,
  VS_FN_LOG = 2,
  VS_FN_EXP = 3,
  VS_FN_SQRT = 4
} vs_math_fn;

/// dst[i] = convert(src[i]); float->int truncates, narrowing saturates.
vs_status vs_convert(const void *src, int src_dtype, void *dst, int dst_dtype,
                     size_t n, vs_stream_t stream);
vs_status vs_binary(int op, const float *a, const float *b, float *out,
                    size_t n, vs_stream_t stream);
/// out = a * b (or a * conj(b)) over n interleaved complex numbers.
vs_status vs_complex_multiply(const float *a, const float *b, float *out,
                              size_t n_complex, int conjugate_b,
                              vs_stream_t stream);
/// Conjugates n_floats/2 interleaved complex numbers (odd tail copied).
vs_status vs_complex_conjugate(const float *a, float *out, size_t n_floats,
                               vs_stream_t stream);
/// out = x * scale + shift.
vs_status vs_affine(const float *x, float scale, float shift, float *out,
                    size_t n, vs_stream_t stream);
/// y = a * x + y.
vs_status vs_saxpy(float a, const float *x, float *y, size_t n,
                   vs_stream_t stream);
vs_status vs_fill(float *dst, float value, size_t n, vs_stream_t stream);
/// dst[i] = src[n-1-i] (complex_pairs: reverse order of float pairs).
vs_status vs_reverse(const float *src, float *dst, size_t n, int complex_pairs,
                     vs_stream_t stream);
vs_status vs_int16_multiply(const int16_t *a, const int16_t *b, int32_t *out,
                            size_t n, vs_stream_t stream);
vs_status vs_math(int fn, const float *x, float *y, size_t n,
                  vs_stream_t stream);
/// out[i] = powf(x[i], y[i]) (reference avx_mathfun.h:720 pow256_ps).
vs_status vs_pow(const float *x, const float *y, float *out, size_t n,
                 vs_stream_t stream);
/// s[i] = sinf(x[i]), c[i] = cosf(x[i]) in one pass (reference
/// avx_mathfun.h:571 sincos256_ps, neon_mathfun.h:228 sincos_ps).
vs_status vs_sincos(const float *x, float *s, float *c, size_t n,
                    vs_stream_t stream);
/// Consumer of <simd/device_math.h> (csrc/kernels/device_math_user.hip, a
/// kernel that includes only that header): morlet[i] = exp(-t^2 / 2)
/// cos(omega t), feature[i] = log(1 + sqrt(|t|^p)).
vs_status vs_device_math_example(const float *t, float omega, float p, size_t n,
                                 float *morlet, float *feature, vs_stream_t stream);

/* ------------------------------------------------------------ reductions */
/// *out_dev = sum(x) (pairwise tree in fp32).
vs_status vs_sum(const float *x, size_t n, float *out_dev, vs_stream_t stream);
/// out_dev[0] = min, out_dev[1] = max.
vs_status vs_minmax(const float *x, size_t n, float *out_dev,
                    vs_stream_t stream);
vs_status vs_minmax2d_u8(const uint8_t *src, int src_stride, int width,
                         int height, uint8_t *out_dev, vs_stream_t stream);
/// `planes` planes `plane_stride` bytes apart in one launch sequence:
/// out_dev[2 p] = min, out_dev[2 p + 1] = max of plane p.
vs_status vs_minmax2d_u8_batched(const uint8_t *src, int src_stride,
                                 int64_t plane_stride, int width, int height,
                                 int planes, uint8_t *out_dev, vs_stream_t stream);
/// If minmax_dev != NULL the bounds are read from it (fused normalize2D),
/// otherwise (vmin, vmax) are used.
vs_status vs_normalize2d_u8(const uint8_t *src, int src_stride, int width,
                            int height, const uint8_t *minmax_dev, int vmin,
                            int vmax, float *dst, int dst_stride,
                            vs_stream_t stream);
/// `planes` planes in one launch; minmax_dev (if not NULL) holds one {min,
/// max} pair per plane (vs_minmax2d_u8_batched), so a stack of images is
/// normalised plane by plane without a host round trip (reference
/// src/normalize.c:445-503, one plane per call).
vs_status vs_normalize2d_u8_batched(const uint8_t *src, int src_stride,
                                    int64_t src_plane_stride, int width, int height,
                                    int planes, const uint8_t *minmax_dev, int vmin,
                                    int vmax, float *dst, int dst_stride,
                                    int64_t dst_plane_stride, vs_stream_t stream);

/* ------------------------------------------------------------------ GEMM */
/// C = alpha * op(A) * op(B) + beta * C, row-major, exact fp32 (MFMA f32).
/// op(A) is M x K, op(B) is K x N.  trans flags: 0 = as stored, 1 = transposed.
vs_status vs_sgemm(int trans_a, int trans_b, int m, int n, int k, float alpha,
                   const float *a, int64_t lda, const float *b, int64_t ldb,
                   float beta, float *c, int64_t ldc, vs_stream_t stream);
vs_status vs_sgemm_strided_batched(int trans_a, int trans_b, int m, int n,
                                   int k, float alpha, const float *a,
                                   int64_t lda, int64_t stride_a,
                                   const float *b, int64_t ldb,
                                   int64_t stride_b, float beta, float *c,
                                   int64_t ldc, int64_t stride_c, int batch,
                                   vs_stream_t stream);

/// Number of SGEMM kernel variants accepted by vs_sgemm_variant.
#define VS_SGEMM_VARIANTS 6
/// Tuning entry point: one explicit SGEMM tile size (every variant takes any
/// transpose, ragged shapes and any alignment).  0: 64x64 tiles (4 waves),
/// 1: 128x128 (8 waves), 2: 256x256 (8 waves, AGPR accumulators; 128x128
/// when an operand is not 16-byte aligned), each with automatic k slicing of
/// the tiles that would under-fill the chip; 3..5: the same tiles, whole
/// tiles only.  vs_sgemm picks tile and slicing from a cost model
/// (csrc/kernels/sgemm.hip plan_units); VELES_SGEMM_VARIANT forces one.
vs_status vs_sgemm_variant(int variant, int trans_a, int trans_b, int m, int n,
                           int k, float alpha, const float *a, int64_t lda,
                           const float *b, int64_t ldb, float beta, float *c,
                           int64_t ldc, vs_stream_t stream);
vs_status vs_sgemm_variant_batched(int variant, int trans_a, int trans_b, int m,
                                   int n, int k, float alpha, const float *a,
                                   int64_t lda, int64_t stride_a, const float *b,
                                   int64_t ldb, int64_t stride_b, float beta,
                                   float *c, int64_t ldc, int64_t stride_c,
                                   int batch, vs_stream_t stream);

/// bf16 matrix-core GEMM: C (fp32) = alpha op(A) op(B) + beta C with A, B
/// bf16 (raw uint16 bit patterns), fp32 accumulation (v_mfma_f32_16x16x32_bf16
/// on the large tiles, v_mfma_f32_32x32x16_bf16 on the 128 x 128 tiles).
vs_status vs_gemm_bf16(int trans_a, int trans_b, int m, int n, int k,
                       float alpha, const uint16_t *a, int64_t lda,
                       const uint16_t *b, int64_t ldb, float beta, float *c,
                       int64_t ldc, vs_stream_t stream);
/// Tuning entry point: explicit bf16 kernel variant (LDS-DMA two-stage;
/// 0: 128x128 tiles, 1: 256x256 (bf16) / 256x128 (bf16x3), both on 32x32x16 MFMAs;
/// 2 / 3: the large / small tiles on 16x16x32 MFMAs (2: the two waves of a SIMD issue
/// their DMA a quarter of a tile apart; 4: 2 without that); -1 auto: 2 once the large
/// tiles fill every CU, else 0).
vs_status vs_gemm_bf16_variant(int variant, int trans_a, int trans_b, int m, int n,
                               int k, float alpha, const uint16_t *a, int64_t lda,
                               const uint16_t *b, int64_t ldb, float beta, float *c,
                               int64_t ldc, vs_stream_t stream);
vs_status vs_gemm_bf16_strided_batched(int trans_a, int trans_b, int m, int n,
                                       int k, float alpha, const uint16_t *a,
                                       int64_t lda, int64_t stride_a,
                                       const uint16_t *b, int64_t ldb,
                                       int64_t stride_b, float beta, float *c,
                                       int64_t ldc, int64_t stride_c,
                                       int batch, vs_stream_t stream);
/// Fast fp32 GEMM ("bf16x3"): fp32 operands split into bf16 hi + lo,
/// C = hi hi + hi lo + lo hi on the bf16 matrix cores (~2^-16 relative
/// error per product instead of 2^-24).  variant as for vs_gemm_bf16_variant.
vs_status vs_sgemm_bf16x3(int trans_a, int trans_b, int m, int n, int k,
                          float alpha, const float *a, int64_t lda,
                          const float *b, int64_t ldb, float beta, float *c,
                          int64_t ldc, int variant, vs_stream_t stream);
vs_status vs_sgemm_bf16x3_strided_batched(int trans_a, int trans_b, int m,
                                          int n, int k, float alpha,
                                          const float *a, int64_t lda,
                                          int64_t stride_a, const float *b,
                                          int64_t ldb, int64_t stride_b,
                                          float beta, float *c, int64_t ldc,
                                          int64_t stride_c, int batch,
                                          vs_stream_t stream);

/* ------------------------------------------------------------------- FFT */
/// Unnormalised complex FFT of `batch` contiguous interleaved signals of n
/// (power of two, 2..2^24) points.  inverse=0: exp(-2 pi i jk/n).
vs_status vs_fft_c2c(const float *in, float *out, int n, int batch,
                     int inverse, vs_stream_t stream);
/// Real forward FFT: n real -> n/2+1 complex (n+2 floats) per signal.
vs_status vs_fft_r2c(const float *in, float *out, int n, int batch,
                     vs_stream_t stream);
/// Real inverse FFT (unnormalised): n/2+1 complex -> n real per signal.
vs_status vs_fft_c2r(const float *in, float *out, int n, int batch,
                     vs_stream_t stream);

/* ----------------------------------------------------------- convolution */
typedef enum {
  VS_CONV_AUTO = 0,
  VS_CONV_DIRECT = 1,
  VS_CONV_FFT = 2,
  VS_CONV_OVERLAP_SAVE = 3
} vs_conv_algo;

/// Batched full linear convolution (correlate=0) or cross-correlation
/// (correlate=1): y[b] (length x_len + h_len - 1, row stride y_stride) of
/// x[b] (stride x_stride) with h[b] (stride h_stride; 0 = one shared filter).
vs_status vs_conv1d(int algo, int correlate, const float *x, int64_t x_len,
                    int64_t x_stride, const float *h, int h_len,
                    int64_t h_stride, float *y, int64_t y_stride, int batch,
                    vs_stream_t stream);
/// Algorithm VS_CONV_AUTO resolves to for this shape.
int vs_conv1d_select(int64_t x_len, int h_len, int batch);
/// Overlap-save block length the library uses for filter length h_len.
int vs_conv1d_os_block(int h_len);

/// Convolution plan: fixed filter(s) and signal length, many executions
/// (FIR filters, matched filters at inference).  Creation resolves the
/// algorithm and, on the real-block FFT / overlap-save paths, computes the
/// filter spectra once (the per-call vs_conv1d recomputes them: ~13 us for a
/// 4096-tap filter); other paths keep a device copy of the taps and run
/// vs_conv1d.  h: n_filters rows of h_len taps, row stride h_stride (device
/// pointer; copied / transformed during creation, on `stream`).
/// n_filters = 1 (shared filter, any batch) or the batch (one per signal).
typedef struct vs_conv_plan vs_conv_plan;
vs_status vs_conv1d_plan_create(int algo, int correlate, int64_t x_len, const float *h,
                                int h_len, int64_t h_stride, int n_filters,
                                vs_conv_plan **plan, vs_stream_t stream);
/// y[b] = x[b] (*) h of the plan; the same contract as vs_conv1d.
vs_status vs_conv1d_plan_execute(const vs_conv_plan *plan, const float *x,
                                 int64_t x_stride, float *y, int64_t y_stride,
                                 int batch, vs_stream_t stream);
/// Resolved algorithm and whether the filter spectra are precomputed.
vs_status vs_conv1d_plan_info(const vs_conv_plan *plan, int *algo, int *precomputed);
/// Frees the plan (after the streams that used it are done with it).
void vs_conv1d_plan_destroy(vs_conv_plan *plan);
/// Tuning knobs for measurements ("os_block_log_max": cap of the
/// overlap-save block, log2).
/// The knobs are per thread: a call changes what later calls of the same
/// thread do, never another thread's; plans keep what they were created with.
vs_status vs_tune_set(const char *key, int value);
/// Restores every knob of the calling thread to its default.
void vs_tune_reset(void);

/* -------------------------------------------------------------- wavelets */
/// Batched single-level decimated DWT: hi/lo rows of len/2 (stride
/// out_stride) per input row (stride src_stride).
vs_status vs_dwt(int type, int order, int ext, const float *src, int64_t len,
                 int64_t src_stride, float *hi, float *lo, int64_t out_stride,
                 int batch, vs_stream_t stream);
/// Batched single-level stationary DWT at `level` (full-length outputs).
vs_status vs_swt(int type, int order, int level, int ext, const float *src,
                 int64_t len, int64_t src_stride, float *hi, float *lo,
                 int64_t out_stride, int batch, vs_stream_t stream);
/// Fused `levels`-level stationary DWT, level l fed by level l-1's lo:
/// hi is [batch][levels][len], lo is [batch][len] (the last level's lo).
vs_status vs_swt_multilevel(int type, int order, int levels, int ext,
                            const float *src, int64_t len, float *hi, float *lo,
                            int batch, vs_stream_t stream);
/// The same transform into one array: out is [batch][levels + 1][len], rows
/// 0 .. levels-1 of a signal its hi bands, row `levels` its low band.  A
/// signal's output is one contiguous block, which the memory system takes
/// ~6 % faster than separate hi and lo arrays (65536 x 1024, 8 levels).
vs_status vs_swt_multilevel_packed(int type, int order, int levels, int ext,
                                   const float *src, int64_t len, float *out,
                                   int batch, vs_stream_t stream);
/// Fused `levels`-level decimated DWT (Mallat pyramid); per row of out
/// (length len): [hi_1 (len/2) | hi_2 (len/4) | ... | hi_L | lo_L].
vs_status vs_dwt_multilevel(int type, int order, int levels, int ext,
                            const float *src, int64_t len, float *out, int batch,
                            vs_stream_t stream);
/// Copies the float low-pass filter (order taps) into host memory `out`.
vs_status vs_wavelet_filter(int type, int order, float *out);

/* ----------------------------------------------------------------- peaks */
/// Ordered strict extrema of x[0..n): positions/values of the first
/// `capacity` go to pos_dev/val_dev, the total count to *count_dev.
vs_status vs_detect_peaks(const float *x, size_t n, int type, int *pos_dev,
                          float *val_dev, size_t capacity,
                          unsigned long long *count_dev, vs_stream_t stream);
/// Extrema of `rows` signals of n samples (x_stride floats apart) in one
/// launch sequence, no host synchronisation: results of all rows back to
/// back in (row, position) order, row r's in
/// [row_start_dev[r], row_start_dev[r + 1]) (rows + 1 entries; the last is
/// the total).  Positions are indices inside the row: int32, or int64 when
/// pos64 != 0 (required for n >= 2^31; the reference's size argument is a
/// size_t, inc/simd/detect_peaks.h:61-62).  Call with capacity 0 to size the
/// outputs, then again with the arrays.
vs_status vs_detect_peaks_batched(const float *x, size_t n, int64_t x_stride, size_t rows,
                                  int type, void *pos_dev, int pos64, float *val_dev,
                                  size_t capacity, unsigned long long *row_start_dev,
                                  vs_stream_t stream);

SIMD_API_END

#endif  // VELES_SIMD_GPU_H_
