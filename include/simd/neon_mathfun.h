/*! @file neon_mathfun.h
 *  @brief sqrt over float arrays, plus the sincos / pow array operations:
 *  the element functions of the reference's 4-lane NEON cephes header.
 *
 *  Reference inc/simd/neon_mathfun.h (3rd-party, Pommier 2011): log_ps
 *  (:57), exp_ps (:142), sincos_ps (:228), sin_ps (:295), cos_ps (:301),
 *  pow_ps (:307) and sqrt_ps (:314-332, four Newton iterations of the
 *  reciprocal square root estimate) on float32x4_t.  As with
 *  <simd/avx_mathfun.h>, the wavefront replaces the register: sqrt_psv is
 *  a correctly rounded square root on the GPU (simd != 0) or libm sqrtf on
 *  the host (simd == 0), i.e. more accurate than the reference's estimate.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_NEON_MATHFUN_H_
#define VELES_SIMD_NEON_MATHFUN_H_

#include <math.h>
#include <stddef.h>
#include <simd/attributes.h>
#include <simd/avx_mathfun.h>
#include <simd/common.h>

SIMD_API_BEGIN

/// res[i] = sqrt(src[i]) (sqrt_ps over an array).
INLINE void sqrt_psv_novec(const float *src, size_t length, float *res) {
  for (size_t i = 0; i < length; ++i) res[i] = sqrtf(src[i]);
}

void sqrt_psv(int simd, const float *src, size_t length, float *res) NOTNULL(2, 4);

SIMD_API_END

#endif  // VELES_SIMD_NEON_MATHFUN_H_
