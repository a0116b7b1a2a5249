/*! @file convolve_structs.h
 *  @brief Convolution handle types (returned by value).
 *
 *  Field-for-field source-compatible with reference
 *  inc/simd/convolve_structs.h:39-74.  As in the reference, the state lives
 *  behind heap pointers, so copies of a handle alias the same plan; the
 *  matching *_finalize releases it.  fft_plan / fft_inverse_plan point to
 *  this library's GPU plan objects (device buffers, twiddles, stream).
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_CONVOLVE_STRUCTS_H_
#define VELES_SIMD_CONVOLVE_STRUCTS_H_

#include <stddef.h>
#include <simd/common.h>

SIMD_API_BEGIN

struct ConvolutionOverlapSaveHandle {
  void *fft_plan;
  void *fft_inverse_plan;
  float *fft_boiler_plate;
  float *H;
  size_t x_length;
  size_t h_length;
  int *L;
  int reverse;
};

struct ConvolutionFFTHandle {
  void *fft_plan;
  void *fft_inverse_plan;
  int *M;
  int x_length;
  int h_length;
  float **inputs;
  int reverse;
};

typedef enum {
  kConvolutionAlgorithmBruteForce,
  kConvolutionAlgorithmFFT,
  kConvolutionAlgorithmOverlapSave
} ConvolutionAlgorithm;

struct ConvolutionHandle {
  ConvolutionAlgorithm algorithm;
  int x_length;
  int h_length;
  union {
    struct ConvolutionFFTHandle fft;
    struct ConvolutionOverlapSaveHandle os;
  } handle;
};

SIMD_API_END

#endif  // VELES_SIMD_CONVOLVE_STRUCTS_H_
