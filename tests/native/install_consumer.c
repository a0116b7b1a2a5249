/* Plain-C consumer of an installed veles.simd_amd (tests/test_install.py):
 * includes every public header of the reference's API, compiles with gcc
 * using only the flags of the installed Simd.pc, and runs host-path calls. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <simd/arithmetic.h>
#include <simd/avx_mathfun.h>
#include <simd/convolve.h>
#include <simd/correlate.h>
#include <simd/detect_peaks.h>
#include <simd/instruction_set.h>
#include <simd/mathfun.h>
#include <simd/matrix.h>
#include <simd/memory.h>
#include <simd/neon_mathfun.h>
#include <simd/normalize.h>
#include <simd/wavelet.h>

int main(void) {
  float x[64], h[5], y[68];
  for (int i = 0; i < 64; i++) x[i] = (float)(i % 7) - 3.f;
  for (int i = 0; i < 5; i++) h[i] = 0.5f * (float)i;
  convolve_simd(0, x, 64, h, 5, y);
  double ref = 0;
  for (int m = 0; m < 5; m++) ref += h[m] * x[10 - m];
  if (fabs(y[10] - ref) > 1e-5) { printf("convolve mismatch %f %f\n", y[10], ref); return 1; }

  float a[6] = {1, 2, 3, 4, 5, 6}, b[6] = {1, 0, 0, 1, 1, 1}, c[4];
  matrix_multiply(0, a, b, 3, 2, 2, 3, c);  /* (2x3) x (3x2) */
  if (c[0] != 4.f || c[3] != 11.f) { printf("matrix mismatch %f %f\n", c[0], c[3]); return 1; }

  float *src = mallocf(16);
  float hi[8], lo[8];
  for (int i = 0; i < 16; i++) src[i] = (float)i;
  wavelet_apply_na(WAVELET_TYPE_DAUBECHIES, 4, EXTENSION_TYPE_PERIODIC, src, 16, hi, lo);
  free(src);
  printf("ok %f %f\n", y[10], lo[0]);
  return 0;
}
