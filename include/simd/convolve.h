/*! @file convolve.h
 *  @brief Full linear 1D convolution: result[n] = sum_m h[m] x[n-m],
 *  n in [0, xLength + hLength - 1).
 *
 *  Source-compatible with reference inc/simd/convolve.h:41-125.  Three
 *  algorithms, each a HIP kernel pipeline on MI355X:
 *   - brute force (convolve_simd): LDS-tiled direct convolution;
 *   - FFT: zero-pad to M = next pow2 >= x+h-1, our own Stockham FFT
 *     (replaces the reference's FFTF dependency), pointwise product, inverse;
 *   - overlap-save: block size L = 2^(floor(log2 h)+2), all blocks of the
 *     signal transformed by ONE fused kernel (LDS-resident FFT -> x H ->
 *     inverse FFT -> store valid samples), instead of the reference's serial
 *     block loop.
 *  convolve_initialize() auto-selects an algorithm with the reference
 *  heuristic (reference src/convolve.c:328-366).  The result always has
 *  length xLength + hLength - 1.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_CONVOLVE_H_
#define VELES_SIMD_CONVOLVE_H_

#include <stddef.h>
#include <simd/attributes.h>
#include <simd/common.h>
#include <simd/convolve_structs.h>

SIMD_API_BEGIN

typedef struct ConvolutionFFTHandle ConvolutionFFTHandle;

ConvolutionFFTHandle convolve_fft_initialize(size_t xLength, size_t hLength);
void convolve_fft(ConvolutionFFTHandle handle, const float *x,
                  const float *h, float *result) NOTNULL(2, 3, 4);
void convolve_fft_finalize(ConvolutionFFTHandle handle);

typedef struct ConvolutionOverlapSaveHandle ConvolutionOverlapSaveHandle;

/// Requires hLength < xLength / 2 (reference src/convolve.c:105).
ConvolutionOverlapSaveHandle convolve_overlap_save_initialize(
    size_t xLength, size_t hLength);
void convolve_overlap_save(ConvolutionOverlapSaveHandle handle,
                           const float *x, const float *h, float *result)
    NOTNULL(2, 3, 4);
void convolve_overlap_save_finalize(ConvolutionOverlapSaveHandle handle);

/// Direct convolution; simd != 0 on the GPU, 0 on the host.
void convolve_simd(int simd, const float *__restrict x, size_t xLength,
                   const float *__restrict h, size_t hLength,
                   float *__restrict result) NOTNULL(2, 4, 6);

typedef struct ConvolutionHandle ConvolutionHandle;

ConvolutionHandle convolve_initialize(size_t xLength, size_t hLength);
void convolve(ConvolutionHandle handle, const float *__restrict x,
              const float *__restrict h, float *__restrict result)
    NOTNULL(2, 3, 4);
void convolve_finalize(ConvolutionHandle handle);

SIMD_API_END

#endif  // VELES_SIMD_CONVOLVE_H_
