/*! @file mathfun.h
 *  @brief Elementwise sin / cos / log / exp over float arrays.
 *
 *  Source-compatible with reference inc/simd/mathfun.h:142-204.  simd != 0
 *  runs the HIP kernel (OCML-accurate transcendental functions, <= 2 ulp
 *  vs. double libm, which beats the reference's cephes polynomials); simd
 *  == 0 runs libm on the host (the *_novec path).  simd != 0 on short host
 *  arrays runs glibc's vector math library on the host (AVX2, at most 4 ulp
 *  off libm) instead of a GPU round trip.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_MATHFUN_H_
#define VELES_SIMD_MATHFUN_H_

#include <math.h>
#include <stddef.h>
#include <simd/attributes.h>
#include <simd/common.h>
#include <simd/instruction_set.h>
/* sincos_psv / pow_psv / sqrt_psv: the reference's avx_mathfun.h /
 * neon_mathfun.h element functions over arrays (reference mathfun.h
 * includes those headers, :30-40). */
#include <simd/neon_mathfun.h>

SIMD_API_BEGIN

typedef float (*PsvStdFunc)(float);

INLINE void func_psv_novec(PsvStdFunc func, const float *src, size_t length,
                           float *res) {
  for (size_t i = 0; i < length; ++i) {
    res[i] = func(src[i]);
  }
}

INLINE void sin_psv_novec(const float *src, size_t length, float *res) {
  func_psv_novec(sinf, src, length, res);
}
INLINE void cos_psv_novec(const float *src, size_t length, float *res) {
  func_psv_novec(cosf, src, length, res);
}
INLINE void log_psv_novec(const float *src, size_t length, float *res) {
  func_psv_novec(logf, src, length, res);
}
INLINE void exp_psv_novec(const float *src, size_t length, float *res) {
  func_psv_novec(expf, src, length, res);
}

void sin_psv(int simd, const float *src, size_t length, float *res)
    NOTNULL(2, 4);
void cos_psv(int simd, const float *src, size_t length, float *res)
    NOTNULL(2, 4);
void log_psv(int simd, const float *src, size_t length, float *res)
    NOTNULL(2, 4);
void exp_psv(int simd, const float *src, size_t length, float *res)
    NOTNULL(2, 4);

SIMD_API_END

#endif  // VELES_SIMD_MATHFUN_H_
