/*! @file device_math.h
 *  @brief Device-callable transcendental math: the register-level functions
 *  of the reference's cephes headers, for composing into user HIP kernels.
 *
 *  The reference's math headers are register-level building blocks that
 *  other code calls from inside its own loops: log256_ps, exp256_ps,
 *  sin256_ps, cos256_ps, sincos256_ps, pow256_ps on 8 AVX lanes
 *  (inc/simd/avx_mathfun.h:161, :247, :327, :454, :571, :720) and log_ps,
 *  exp_ps, sincos_ps, sin_ps, cos_ps, pow_ps, sqrt_ps on 4 NEON lanes
 *  (inc/simd/neon_mathfun.h:57-332).  On the GPU the register is a 64-lane
 *  wavefront and a kernel is written per lane, so the same building blocks
 *  are per-lane __device__ functions (and float4 forms for kernels that move
 *  16 bytes per lane).  They are the functions the library's own array
 *  kernels (<simd/mathfun.h>, <simd/avx_mathfun.h>, <simd/neon_mathfun.h>)
 *  are built from: every result is within 4 ulp of double-precision libm
 *  (exp, sqrt, pow within 1), the bound the reference's tests use
 *  (tests/mathfun.cc:59-73).
 *
 *  Include from HIP device code (hipcc, gfx950):
 *    __global__ void k(const float *x, float *y, size_t n) {
 *      size_t i = blockIdx.x * blockDim.x + threadIdx.x;
 *      if (i < n) y[i] = simd_exp_ps(-0.5f * x[i] * x[i]) * simd_cos_ps(x[i]);
 *    }
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_DEVICE_MATH_H_
#define VELES_SIMD_DEVICE_MATH_H_

#include <hip/hip_runtime.h>

/// exp(x): two-constant (Cody-Waite) reduction x = n ln2 + r, a degree-7
/// polynomial on |r| <= ln2 / 2, then ldexp; <= 1 ulp over the whole range
/// (exp2(x log2 e) loses |x| 2^-24 relative accuracy in the product, up to
/// ~40 ulp near x = 88).  Overflow gives +inf, underflow 0, NaN propagates.
__device__ __forceinline__ float simd_exp_ps(float x) {
  if (!(x < 88.72283935546875f)) return x != x ? x : __builtin_inff();
  if (x < -103.97208404541015625f) return 0.f;
  const float n = rintf(x * 1.44269504088896341f);
  float r = fmaf(n, -0.693145751953125f, x);
  r = fmaf(n, -1.428606765330187045e-6f, r);
  float p = 1.98412698412698413e-4f;
  p = fmaf(p, r, 1.38888888888888889e-3f);
  p = fmaf(p, r, 8.33333333333333333e-3f);
  p = fmaf(p, r, 4.16666666666666667e-2f);
  p = fmaf(p, r, 1.66666666666666667e-1f);
  p = fmaf(p, r, 0.5f);
  p = fmaf(p, r, 1.0f);
  p = fmaf(p, r, 1.0f);
  return ldexpf(p, static_cast<int>(n));
}

/// log(x) (natural); negative arguments give NaN, 0 gives -inf.
__device__ __forceinline__ float simd_log_ps(float x) { return logf(x); }
/// sin(x), any x (full-range argument reduction).
__device__ __forceinline__ float simd_sin_ps(float x) { return sinf(x); }
/// cos(x), any x.
__device__ __forceinline__ float simd_cos_ps(float x) { return cosf(x); }
/// sin and cos of the same argument with one shared range reduction.
__device__ __forceinline__ void simd_sincos_ps(float x, float *s, float *c) { sincosf(x, s, c); }
/// sqrt(x), correctly rounded (the reference's NEON form is four
/// Newton-Raphson rsqrt steps: neon_mathfun.h:314-332).
__device__ __forceinline__ float simd_sqrt_ps(float x) { return sqrtf(x); }
/// x^y, evaluated in double and rounded once: <= 1 ulp (a float powf was
/// measured at up to 5 ulp, 15.65^4.2).
__device__ __forceinline__ float simd_pow_ps(float x, float y) {
  return static_cast<float>(pow(static_cast<double>(x), static_cast<double>(y)));
}

/// 4-lane forms for kernels that load and store one float4 per lane.
#define SIMD_DEVICE_MATH_V4(NAME)                                                  \
  __device__ __forceinline__ float4 NAME##4(float4 v) {                            \
    return make_float4(NAME(v.x), NAME(v.y), NAME(v.z), NAME(v.w));                \
  }
SIMD_DEVICE_MATH_V4(simd_exp_ps)
SIMD_DEVICE_MATH_V4(simd_log_ps)
SIMD_DEVICE_MATH_V4(simd_sin_ps)
SIMD_DEVICE_MATH_V4(simd_cos_ps)
SIMD_DEVICE_MATH_V4(simd_sqrt_ps)
#undef SIMD_DEVICE_MATH_V4
__device__ __forceinline__ void simd_sincos_ps4(float4 v, float4 *s, float4 *c) {
  simd_sincos_ps(v.x, &s->x, &c->x);
  simd_sincos_ps(v.y, &s->y, &c->y);
  simd_sincos_ps(v.z, &s->z, &c->z);
  simd_sincos_ps(v.w, &s->w, &c->w);
}
__device__ __forceinline__ float4 simd_pow_ps4(float4 x, float4 y) {
  return make_float4(simd_pow_ps(x.x, y.x), simd_pow_ps(x.y, y.y), simd_pow_ps(x.z, y.z),
                     simd_pow_ps(x.w, y.w));
}

#endif  // VELES_SIMD_DEVICE_MATH_H_
