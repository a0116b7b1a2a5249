/*! @file matrix.h
 *  @brief Row-major float matrix add / sub / GEMM ("parts of BLAS").
 *
 *  Source-compatible with reference inc/simd/matrix.h:47-89.  simd != 0
 *  runs on the GPU: add/sub as a vectorised elementwise kernel, the two
 *  products as the MFMA fp32 SGEMM (v_mfma_f32_32x32x2_f32, exact fp32).
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_MATRIX_H_
#define VELES_SIMD_MATRIX_H_

#include <stddef.h>
#include <simd/attributes.h>
#include <simd/common.h>

SIMD_API_BEGIN

/// res = m1 + m2, both w x h (w = row length).
void matrix_add(int simd, const float *m1, const float *m2, size_t w,
                size_t h, float *res) NOTNULL(2, 3, 6);
/// res = m1 - m2.
void matrix_sub(int simd, const float *m1, const float *m2, size_t w,
                size_t h, float *res) NOTNULL(2, 3, 6);
/// res[h1 x w2] = m1[h1 x w1] * m2[h2 x w2]; requires w1 == h2.
void matrix_multiply(int simd, const float *m1, const float *m2, size_t w1,
                     size_t h1, size_t w2, size_t h2, float *res)
    NOTNULL(2, 3, 8);
/// res[h1 x h2] = m1[h1 x w1] * transpose(m2[h2 x w2]); requires w1 == w2.
void matrix_multiply_transposed(int simd, const float *m1, const float *m2,
                                size_t w1, size_t h1, size_t w2, size_t h2,
                                float *res) NOTNULL(2, 3, 8);

SIMD_API_END

#endif  // VELES_SIMD_MATRIX_H_
