/*! @file correlate.h
 *  @brief Full cross-correlation:
 *  result[k] = sum_m x[m] h[m + hLength - 1 - k], k in [0, x+h-1).
 *
 *  Source-compatible with reference inc/simd/correlate.h:41-135.  The FFT
 *  and overlap-save variants are convolution with h reversed (the reversal is
 *  folded into the filter upload, reference src/convolve.c:167-171), the
 *  brute-force variant is its own GPU kernel.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_CORRELATE_H_
#define VELES_SIMD_CORRELATE_H_

#include <stddef.h>
#include <simd/attributes.h>
#include <simd/common.h>
#include <simd/convolve_structs.h>

SIMD_API_BEGIN

typedef struct ConvolutionFFTHandle CrossCorrelationFFTHandle;

CrossCorrelationFFTHandle cross_correlate_fft_initialize(size_t xLength,
                                                         size_t hLength);
void cross_correlate_fft(CrossCorrelationFFTHandle handle, const float *x,
                         const float *h, float *result) NOTNULL(2, 3, 4);
void cross_correlate_fft_finalize(CrossCorrelationFFTHandle handle);

typedef struct ConvolutionOverlapSaveHandle CrossCorrelationOverlapSaveHandle;

CrossCorrelationOverlapSaveHandle cross_correlate_overlap_save_initialize(
    size_t xLength, size_t hLength);
void cross_correlate_overlap_save(CrossCorrelationOverlapSaveHandle handle,
                                  const float *__restrict x,
                                  const float *__restrict h, float *result)
    NOTNULL(2, 3, 4);
void cross_correlate_overlap_save_finalize(
    CrossCorrelationOverlapSaveHandle handle);

void cross_correlate_simd(int simd, const float *__restrict x,
                          size_t xLength, const float *__restrict h,
                          size_t hLength, float *__restrict result)
    NOTNULL(2, 4, 6);

typedef struct ConvolutionHandle CrossCorrelationHandle;

CrossCorrelationHandle cross_correlate_initialize(size_t xLength,
                                                  size_t hLength);
void cross_correlate(CrossCorrelationHandle handle,
                     const float *__restrict x, const float *__restrict h,
                     float *__restrict result) NOTNULL(2, 3, 4);
void cross_correlate_finalize(CrossCorrelationHandle handle);

SIMD_API_END

#endif  // VELES_SIMD_CORRELATE_H_
