/*! @file avx_mathfun.h
 *  @brief sincos / pow over float arrays: the element functions of the
 *  reference's 8-lane cephes header as whole-array operations.
 *
 *  The reference header (inc/simd/avx_mathfun.h, 3rd-party, Garberoglio
 *  2012) defines register-level AVX functions: log256_ps (:161),
 *  exp256_ps (:247), sin256_ps (:327), cos256_ps (:454), sincos256_ps
 *  (:571) and pow256_ps (:720) on __m256.  There is no host SIMD path in
 *  this library: a 64-lane wavefront replaces the 8-lane
 *  register, so the same functions are offered over arrays, evaluated on the
 *  GPU for simd != 0 (OCML sincosf; pow evaluated in double and rounded once,
 *  <= 1 ulp against double)
 *  and by libm on the host for simd == 0 (the *_novec twins below).
 *  log / exp / sin / cos over arrays are in <simd/mathfun.h>.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_AVX_MATHFUN_H_
#define VELES_SIMD_AVX_MATHFUN_H_

#include <math.h>
#include <stddef.h>
#include <simd/attributes.h>
#include <simd/common.h>

SIMD_API_BEGIN

/// s[i] = sin(src[i]), c[i] = cos(src[i]) (sincos256_ps over an array).
INLINE void sincos_psv_novec(const float *src, size_t length, float *s, float *c) {
  for (size_t i = 0; i < length; ++i) {
    s[i] = sinf(src[i]);
    c[i] = cosf(src[i]);
  }
}

/// res[i] = x[i] ^ y[i] (pow256_ps over arrays).
INLINE void pow_psv_novec(const float *x, const float *y, size_t length, float *res) {
  for (size_t i = 0; i < length; ++i) res[i] = powf(x[i], y[i]);
}

void sincos_psv(int simd, const float *src, size_t length, float *s, float *c)
    NOTNULL(2, 4, 5);
void pow_psv(int simd, const float *x, const float *y, size_t length, float *res)
    NOTNULL(2, 3, 5);

SIMD_API_END

#endif  // VELES_SIMD_AVX_MATHFUN_H_
