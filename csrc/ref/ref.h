// CPU scalar reference implementations (namespace vs::ref).
//
// These encode the reference library's scalar semantics (its *_na / *_novec
// bodies) and serve two roles: the `simd == 0` path of the public API, and
// the oracle every GPU kernel is tested against.  They are deliberately
// plain loops; there is no CPU-SIMD path in this library.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#pragma once

#include <cstddef>
#include <cstdint>

#include "simd/detect_peaks.h"
#include "simd/wavelet_types.h"

namespace vs {
namespace ref {

// matrix.c scalar bodies (reference src/matrix.c:37-80).
void matrix_add(const float *a, const float *b, size_t w, size_t h,
                float *res);
void matrix_sub(const float *a, const float *b, size_t w, size_t h,
                float *res);
void matrix_multiply(const float *a, const float *b, size_t w1, size_t h1,
                     size_t w2, float *res);
void matrix_multiply_transposed(const float *a, const float *b, size_t w1,
                                size_t h1, size_t h2, float *res);

// Direct convolution / cross-correlation (reference src/convolve.c:40-101,
// src/correlate.c:74-126), full length x + h - 1.
void convolve_direct(const float *x, size_t xl, const float *h, size_t hl,
                     float *y);
void correlate_direct(const float *x, size_t xl, const float *h, size_t hl,
                      float *y);
// FFT-based linear convolution on the host (double-precision radix-2 FFT);
// used when no GPU is present for the FFT / overlap-save handles.
void convolve_fft(const float *x, size_t xl, const float *h, size_t hl,
                  int reverse_h, float *y);
// In-place complex FFT of n (power of two) interleaved doubles.
void fft_inplace(double *data, size_t n, bool inverse);

// normalize.c scalar bodies (reference src/normalize.c:382-443).
void minmax2d(const uint8_t *src, int stride, int w, int h, uint8_t *mn,
              uint8_t *mx);
void normalize2d_minmax(uint8_t mn, uint8_t mx, const uint8_t *src,
                        int sstride, int w, int h, float *dst, int dstride);
void minmax1d(const float *src, int n, float *mn, float *mx);

// detect_peaks scalar definition (reference src/detect_peaks.c:41-56,
// :123-125); returns a malloc()'d array.
void detect_peaks(const float *x, size_t n, ExtremumType type,
                  ExtremumPoint **out, size_t *count);

// Wavelets (reference src/wavelet.c:271-382).
void dwt(WaveletType type, int order, ExtensionType ext, const float *src,
         size_t len, float *hi, float *lo);
void swt(WaveletType type, int order, int level, ExtensionType ext,
         const float *src, size_t len, float *hi, float *lo);

}  // namespace ref

// Vectorised host paths for tiny calls (csrc/ref/host_fast.cpp): the same
// sums as the scalar reference above, unit-stride inner loops.
namespace host {
void convolve_direct(const float *x, size_t xl, const float *h, size_t hl, float *y);
void correlate_direct(const float *x, size_t xl, const float *h, size_t hl, float *y);
void dwt(WaveletType type, int order, ExtensionType ext, const float *src, size_t len,
         float *hi, float *lo);
void swt(WaveletType type, int order, int level, ExtensionType ext, const float *src,
         size_t len, float *hi, float *lo);
bool vector_math(int fn, const float *x, const float *y, size_t n, float *res);
bool has_vector_math();
float sum_elements(const float *a, size_t n);
void minmax1d(const float *src, size_t n, float *mn, float *mx);
void detect_peaks(const float *x, size_t n, ExtremumType type, ExtremumPoint **out,
                  size_t *count);
void matrix_add(const float *a, const float *b, size_t w, size_t h, float *res);
void matrix_sub(const float *a, const float *b, size_t w, size_t h, float *res);
void matrix_multiply(const float *a, const float *b, size_t w1, size_t h1, size_t w2,
                     float *res);
void matrix_multiply_transposed(const float *a, const float *b, size_t w1, size_t h1,
                                size_t h2, float *res);
}  // namespace host
}  // namespace vs
