/* The reference's convolution API, unchanged: build against the installed
 * headers and library (`make install PREFIX=...`), e.g.
 *   cc convolve_demo.c $(pkg-config --cflags --libs Simd) -lm -o convolve_demo
 * A 100,000-sample signal is filtered with 257 taps three ways: the
 * auto-selecting handle, the explicit overlap-save handle and the direct sum
 * (simd = 0: the scalar host reference).  With a GPU the first two run the HIP
 * kernels; without one every call runs on the host.
 * Reference API: inc/simd/convolve.h:40-111. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <simd/convolve.h>

int main(void) {
  const size_t xn = 100000, hn = 257;
  float *x = malloc(xn * sizeof(float)), *h = malloc(hn * sizeof(float));
  float *y0 = malloc((xn + hn - 1) * sizeof(float)), *y1 = malloc((xn + hn - 1) * sizeof(float));
  for (size_t i = 0; i < xn; i++) x[i] = sinf(0.01f * (float)i) + 0.25f * sinf(1.7f * (float)i);
  for (size_t i = 0; i < hn; i++) h[i] = 1.0f / (float)hn; /* moving average */

  convolve_simd(0, x, xn, h, hn, y0); /* scalar reference */

  ConvolutionHandle handle = convolve_initialize(xn, hn); /* picks the algorithm */
  convolve(handle, x, h, y1);
  convolve_finalize(handle);
  float err = 0.f;
  for (size_t i = 0; i < xn + hn - 1; i++) err = fmaxf(err, fabsf(y1[i] - y0[i]));
  printf("auto handle        max |diff| vs scalar: %g\n", err);

  ConvolutionOverlapSaveHandle os = convolve_overlap_save_initialize(xn, hn);
  convolve_overlap_save(os, x, h, y1);
  convolve_overlap_save_finalize(os);
  err = 0.f;
  for (size_t i = 0; i < xn + hn - 1; i++) err = fmaxf(err, fabsf(y1[i] - y0[i]));
  printf("overlap-save       max |diff| vs scalar: %g\n", err);

  free(x), free(h), free(y0), free(y1);
  return err < 1e-3f ? 0 : 1;
}
