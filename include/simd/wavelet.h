/*! @file wavelet.h
 *  @brief Decimated and stationary (a trous) discrete wavelet transforms.
 *
 *  Source-compatible with reference inc/simd/wavelet.h:55-161.
 *   - wavelet_apply: one decimated level,
 *       desthi[k] = sum_j hp[j] s~[2k+j], destlo[k] = sum_j lp[j] s~[2k+j],
 *     k < length/2, s~ = src extended past its end by `ext`;
 *   - stationary_wavelet_apply: level l uses the filters dilated by
 *     2^(l-1) and produces full-length outputs.
 *  The accelerated versions are HIP kernels that touch only the `order`
 *  non-zero taps per output; *_na are the host reference.  Device-resident
 *  batched and fused multi-level variants are in simd/gpu.h.
 *
 *  "Prepared arrays": the reference's AVX path needs shifted copies of the
 *  source (reference src/wavelet.c:54-119).  The GPU needs no such layout, so
 *  wavelet_prepare_array() returns an aligned copy (the same contract as the
 *  reference's non-AVX build) and wavelet_allocate_destination() returns
 *  sourceLength/2 floats.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_WAVELET_H_
#define VELES_SIMD_WAVELET_H_

#include <stddef.h>
#include <simd/attributes.h>
#include <simd/common.h>
#include <simd/wavelet_types.h>

SIMD_API_BEGIN

/// 1 if `order` is supported for `type`: Daubechies / Symlet even <= 76,
/// Coiflet multiple of 6 <= 30.
int wavelet_validate_order(WaveletType type, int order);

float *wavelet_prepare_array(int order, const float *src, size_t length)
    NOTNULL(2) MALLOC WARN_UNUSED_RESULT;

float *wavelet_allocate_destination(int order, size_t sourceLength)
    MALLOC WARN_UNUSED_RESULT;

/// Carves four quarter-length buffers out of src (for the next level's
/// hi-hi / hi-lo / lo-hi / lo-lo outputs); NULLs if length % 4 != 0.
void wavelet_recycle_source(int order, float *src, size_t length,
                            float **desthihi, float **desthilo,
                            float **destlohi, float **destlolo)
    NOTNULL(2, 4, 5, 6, 7);

void wavelet_apply(WaveletType type, int order, ExtensionType ext,
                   const float *__restrict src, size_t length,
                   float *__restrict desthi, float *__restrict destlo)
    NOTNULL(4, 6, 7);

void wavelet_apply_na(WaveletType type, int order, ExtensionType ext,
                      const float *__restrict src, size_t length,
                      float *__restrict desthi, float *__restrict destlo)
    NOTNULL(4, 6, 7);

void stationary_wavelet_apply(WaveletType type, int order, int level,
                              ExtensionType ext, const float *__restrict src,
                              size_t length, float *__restrict desthi,
                              float *__restrict destlo) NOTNULL(5, 7, 8);

void stationary_wavelet_apply_na(WaveletType type, int order, int level,
                                 ExtensionType ext,
                                 const float *__restrict src, size_t length,
                                 float *__restrict desthi,
                                 float *__restrict destlo) NOTNULL(5, 7, 8);

SIMD_API_END

#endif  // VELES_SIMD_WAVELET_H_
