/*! @file normalize.h
 *  @brief Min/max search and [-1, 1] normalisation of uint8 planes / floats.
 *
 *  Source-compatible with reference inc/simd/normalize.h:48-90.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_NORMALIZE_H_
#define VELES_SIMD_NORMALIZE_H_

#include <stdint.h>
#include <simd/attributes.h>
#include <simd/common.h>

SIMD_API_BEGIN

/// dst = (src - min) / ((max - min) / 2) - 1 with min/max of src.
void normalize2D(int simd, const uint8_t *src, int src_stride, int width,
                 int height, float *dst, int dst_stride) NOTNULL(2, 6);
/// min / max of a strided uint8 plane; either output pointer may be NULL.
void minmax2D(int simd, const uint8_t *src, int src_stride, int width,
              int height, uint8_t *min, uint8_t *max) NOTNULL(2);
/// Affine map to [-1, 1]; all zeros (row by row, honouring dst_stride) if
/// max == min.
void normalize2D_minmax(int simd, uint8_t min, uint8_t max,
                        const uint8_t *src, int src_stride, int width,
                        int height, float *dst, int dst_stride)
    NOTNULL(4, 8);
/// min / max of a float array; either output pointer may be NULL.
void minmax1D(int simd, const float *src, int length, float *min,
              float *max) NOTNULL(2);

SIMD_API_END

#endif  // VELES_SIMD_NORMALIZE_H_
