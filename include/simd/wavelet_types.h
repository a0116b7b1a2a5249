/*! @file wavelet_types.h
 *  @brief Wavelet family and boundary-extension enums
 *  (reference inc/simd/wavelet_types.h:38-53).
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_WAVELET_TYPES_H_
#define VELES_SIMD_WAVELET_TYPES_H_

#include <simd/common.h>

SIMD_API_BEGIN

typedef enum {
  WAVELET_TYPE_DAUBECHIES,
  WAVELET_TYPE_COIFLET,
  WAVELET_TYPE_SYMLET
} WaveletType;

typedef enum {
  EXTENSION_TYPE_PERIODIC,
  EXTENSION_TYPE_MIRROR,
  EXTENSION_TYPE_CONSTANT,
  EXTENSION_TYPE_ZERO,
} ExtensionType;

SIMD_API_END

#endif  // VELES_SIMD_WAVELET_TYPES_H_
