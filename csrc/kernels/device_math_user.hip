// A kernel written the way a user of <simd/device_math.h> writes one: it
// includes nothing of the library but that public header and composes its
// per-lane functions -- here a Morlet / Gabor atom and a log-power feature,
// the kind of expression the reference's register-level functions
// (inc/simd/avx_mathfun.h exp256_ps / cos256_ps / log256_ps / pow256_ps,
// inc/simd/neon_mathfun.h sqrt_ps) were composed into inside caller loops.
// It doubles as the build-time and run-time check that the header is
// self-contained device code.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <simd/device_math.h>

#include <cstddef>

#include "simd/gpu.h"

namespace {

// morlet[i] = exp(-t^2 / 2) cos(omega t),  feature[i] = log(1 + sqrt(|t|^p))
__global__ __launch_bounds__(256) void morlet_kernel(const float *__restrict__ t, float omega,
                                                     float p, size_t n,
                                                     float *__restrict__ morlet,
                                                     float *__restrict__ feature) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride) {
    const float x = t[i];
    float s, c;
    simd_sincos_ps(omega * x, &s, &c);
    morlet[i] = simd_exp_ps(-0.5f * x * x) * c;
    feature[i] = simd_log_ps(1.f + simd_sqrt_ps(simd_pow_ps(fabsf(x), p)));
  }
}

}  // namespace

extern "C" vs_status vs_device_math_example(const float *t, float omega, float p, size_t n,
                                            float *morlet, float *feature, vs_stream_t stream) {
  if (n == 0) return VS_OK;
  if (!t || !morlet || !feature) return VS_ERR_INVALID;
  const unsigned blocks = static_cast<unsigned>((n + 255) / 256 < 65536 ? (n + 255) / 256 : 65536);
  hipLaunchKernelGGL(morlet_kernel, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     t, omega, p, n, morlet, feature);
  return hipGetLastError() == hipSuccess ? VS_OK : VS_ERR_HIP;
}
