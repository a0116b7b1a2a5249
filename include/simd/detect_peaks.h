/*! @file detect_peaks.h
 *  @brief Strict local extrema of a 1D signal.
 *
 *  Source-compatible with reference inc/simd/detect_peaks.h:40-63.  A point
 *  i in [1, size-2] is an extremum when (x[i]-x[i-1]) * (x[i]-x[i+1]) > 0
 *  (reference src/detect_peaks.c:41-56).  Results are in increasing position
 *  order in a malloc()'d array the caller free()s.  The GPU path is flag ->
 *  wavefront prefix scan -> ordered compaction.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_DETECT_PEAKS_H_
#define VELES_SIMD_DETECT_PEAKS_H_

#include <stddef.h>
#include <simd/attributes.h>
#include <simd/common.h>

SIMD_API_BEGIN

typedef enum {
  kExtremumTypeMaximum = 1,
  kExtremumTypeMinimum,
  kExtremumTypeBoth
} ExtremumType;

typedef struct {
  int position;
  float value;
} ExtremumPoint;

void detect_peaks(int simd, const float *data, size_t size, ExtremumType type,
                  ExtremumPoint **results, size_t *resultsLength)
    NOTNULL(2, 5, 6);

SIMD_API_END

#endif  // VELES_SIMD_DETECT_PEAKS_H_
