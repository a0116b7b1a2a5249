// Native C API test: compiles against include/simd/*.h exactly as a user of
// the reference would (source compatibility) and re-checks the reference's
// golden vectors (tests/*.cc of the reference) through the public symbols.
// Runs host paths everywhere and the GPU paths when a device is visible.
// Usage: capi_test [--list] [name-substring]
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include <simd/arithmetic.h>
#include <simd/convolve.h>
#include <simd/correlate.h>
#include <simd/detect_peaks.h>
#include <simd/gpu.h>
#include <simd/mathfun.h>
#include <simd/matrix.h>
#include <simd/memory.h>
#include <simd/normalize.h>
#include <simd/wavelet.h>

#include "mini_test.h"

TEST_CASE(memory_align_complement) {
  alignas(32) float f[32];
  alignas(32) int16_t s[32];
  CHECK_EQ(0, align_complement_f32(f));
  CHECK_EQ(7, align_complement_f32(&f[1]));
  CHECK_EQ(1, align_complement_f32(&f[7]));
  CHECK_EQ(15, align_complement_i16(&s[1]));
  CHECK_EQ(0, align_complement_i16(&s[16]));
}

TEST_CASE(memory_alloc_and_pad) {
  void *p = malloc_aligned(100);
  CHECK_EQ(0u, reinterpret_cast<uintptr_t>(p) % 64);
  free(p);
  char *q = static_cast<char *>(malloc_aligned_offset(100, 3));
  CHECK_EQ(3u, reinterpret_cast<uintptr_t>(q) % 64);
  free(q - 3);
  float orig[100];
  memsetf(orig, 1.f, 100);
  size_t nl = 0;
  float *z = zeropadding(orig, 100, &nl);
  CHECK_EQ(256u, nl);
  for (int i = 0; i < 100; i++) CHECK_EQ(1.f, z[i]);
  for (int i = 100; i < 256; i++) CHECK_EQ(0.f, z[i]);
  free(z);
  float src[25], dst[25];
  for (int i = 0; i < 25; i++) src[i] = i;
  rmemcpyf(dst + 1, src + 1, 24);
  for (int i = 1; i < 25; i++) CHECK_EQ(dst[i], src[25 - i]);
}

TEST_CASE(arithmetic_goldens) {
  float a[8] = {1, 2, 3, 4, 5, 6, 7, 8};
  float b[8] = {-1.5f, 1, 3.5f, 3, -5.5f, 6.5f, 2, -9};
  float r[8], v[8];
  complex_multiply(a, b, r);
  for (int i = 0; i < 8; i += 2) complex_multiply_na(a + i, b + i, v + i);
  CHECK(memcmp(r, v, sizeof(r)) == 0);
  uint16_t h[] = {12288, 16777, 18103, 49820};
  float hf[4];
  float16_to_float(h, 4, hf);
  CHECK_NEAR(0.125f, hf[0], 1e-6);
  CHECK_NEAR(2.76757812f, hf[1], 1e-5);
  CHECK_NEAR(-3.3046875f, hf[3], 1e-5);
  CHECK_EQ(128, next_highest_power_of_2(100));
}

TEST_CASE(matrix_multiply_golden) {
  const float m1[6] = {1, 2, 3, -2, 0, 4};
  const float m2[12] = {0, 1, 3, -2, 5, -1, 2, 4, -3, 0, -4, 2};
  const float valid[8] = {1, -1, -5, 12, -12, -2, -22, 12};
  for (int simd = 0; simd < 2; simd++) {
    float res[8];
    matrix_multiply(simd, m1, m2, 3, 2, 4, 3, res);
    for (int i = 0; i < 8; i++) CHECK_NEAR(valid[i], res[i], 0.01);
  }
}

TEST_CASE(matrix_multiply_odd_vs_scalar) {
  // tests/matrix.cc: 299x125 * 125x999 (odd everything), tolerance 0.1
  const int w1 = 125, h1 = 299, w2 = 999;
  std::vector<float> m1(w1 * h1), m2(w2 * w1), r0(h1 * w2), r1(h1 * w2);
  for (int i = 0; i < h1; i++)
    for (int j = 0; j < w1; j++) m1[i * w1 + j] = -j % 17 + i % 6;
  for (int i = 0; i < w1; i++)
    for (int j = 0; j < w2; j++) m2[i * w2 + j] = j % 15 - i % 5;
  matrix_multiply(0, m1.data(), m2.data(), w1, h1, w2, w1, r0.data());
  matrix_multiply(1, m1.data(), m2.data(), w1, h1, w2, w1, r1.data());
  for (size_t i = 0; i < r0.size(); i++) CHECK_NEAR(r0[i], r1[i], 0.1);
}

TEST_CASE(normalize_golden) {
  for (int simd = 0; simd < 2; simd++) {
    std::vector<uint8_t> src(128 * 100, 1);
    src[0] = 127;
    src[1] = 15;
    src[10] = 252;
    src[89] = 31;
    src[128 + 21] = 3;
    std::vector<float> dst(100 * 100);
    normalize2D(simd, src.data(), 128, 100, 100, dst.data(), 100);
    CHECK_NEAR(2.f * (127 - 1) / 251 - 1, dst[0], 1e-6);
    CHECK_NEAR(-1.f, dst[2], 1e-7);
    CHECK_NEAR(1.f, dst[10], 1e-7);
    CHECK_NEAR(2.f * (3 - 1) / 251 - 1, dst[121], 1e-6);
  }
}

TEST_CASE(normalize_pieces) {
  std::vector<uint8_t> src(128 * 100, 1);
  src[0] = 127;
  src[10] = 252;
  for (int simd = 0; simd < 2; simd++) {
    uint8_t mn = 0, mx = 0;
    minmax2D(simd, src.data(), 128, 100, 100, &mn, &mx);
    CHECK_EQ(1, mn);
    CHECK_EQ(252, mx);
    std::vector<float> dst(100 * 100, 7.f);
    normalize2D_minmax(simd, 1, 252, src.data(), 128, 100, 100, dst.data(), 100);
    CHECK_NEAR(-1.f, dst[2], 1e-7);
    CHECK_NEAR(1.f, dst[10], 1e-7);
    if (dst[10] != 1.f)
      std::printf("  simd=%d gpu=%d dst[0..3]=%g %g %g %g err='%s'\n", simd,
                  vs_gpu_available(), dst[0], dst[1], dst[2], dst[3],
                  vs_last_error());
  }
}

TEST_CASE(mathfun_vs_double) {
  const int n = 199;
  float x[n], y[n];
  for (int i = 0; i < n; i++) x[i] = (float(i % 19) - float(i % 6)) * 1.1f;
  for (int simd = 0; simd < 2; simd++) {
    sin_psv(simd, x, n, y);
    for (int i = 0; i < n; i++)
      CHECK_NEAR(static_cast<float>(std::sin(double(x[i]))), y[i], 4e-7);
    exp_psv(simd, x, n, y);
    for (int i = 0; i < n; i++) {
      // ASSERT_FLOAT_EQ semantics: within 4 ulp of the rounded double result
      const float e = static_cast<float>(std::exp(double(x[i])));
      CHECK_NEAR(e, y[i], 4.0 * std::nextafter(std::fabs(e), INFINITY) -
                              4.0 * std::fabs(e));
    }
  }
}

// reference tests/convolve.cc:53-71 and tests/correlate.cc:53-71
TEST_CASE(convolve_correlate_goldens) {
  const float x[8] = {1, 2, 3, 4, 5, 6, 7, 8}, h[4] = {10, 9, 8, 7};
  const float conv[11] = {10, 29, 56, 90, 124, 158, 192, 226, 170, 113, 56};
  const float corr[11] = {7, 22, 46, 80, 114, 148, 182, 216, 187, 142, 80};
  float y[11];
  for (int simd = 0; simd < 2; simd++) {
    convolve_simd(simd, x, 8, h, 4, y);
    for (int i = 0; i < 11; i++) CHECK_NEAR(conv[i], y[i], 1e-4);
    cross_correlate_simd(simd, x, 8, h, 4, y);
    for (int i = 0; i < 11; i++) CHECK_NEAR(corr[i], y[i], 1e-4);
  }
  // every algorithm through the auto-selecting handle API
  ConvolutionHandle hc = convolve_initialize(8, 4);
  convolve(hc, x, h, y);
  for (int i = 0; i < 11; i++) CHECK_NEAR(conv[i], y[i], 1e-3);
  convolve_finalize(hc);
}

// reference tests/convolve.cc:73-137: FFT and overlap-save vs brute force
TEST_CASE(convolve_fft_overlap_save_vs_brute) {
  const int xl = 1021, hl = 50;
  std::vector<float> x(xl), h(hl), ref(xl + hl - 1), y(xl + hl - 1);
  for (int i = 0; i < xl; i++) x[i] = std::sin(static_cast<float>(i)) * 100;
  for (int i = 0; i < hl; i++) h[i] = i / (hl - 1.f);
  convolve_simd(0, x.data(), xl, h.data(), hl, ref.data());
  ConvolutionFFTHandle f = convolve_fft_initialize(xl, hl);
  convolve_fft(f, x.data(), h.data(), y.data());
  convolve_fft_finalize(f);
  for (int i = 0; i < xl + hl - 1; i++) CHECK_NEAR(ref[i], y[i], 1e-3);
  ConvolutionOverlapSaveHandle o = convolve_overlap_save_initialize(xl, hl);
  convolve_overlap_save(o, x.data(), h.data(), y.data());
  convolve_overlap_save_finalize(o);
  for (int i = 0; i < xl + hl - 1; i++) CHECK_NEAR(ref[i], y[i], 1e-3);
  CrossCorrelationFFTHandle cf = cross_correlate_fft_initialize(xl, hl);
  cross_correlate_fft(cf, x.data(), h.data(), y.data());
  cross_correlate_fft_finalize(cf);
  cross_correlate_simd(0, x.data(), xl, h.data(), hl, ref.data());
  for (int i = 0; i < xl + hl - 1; i++) CHECK_NEAR(ref[i], y[i], 1e-3);
}

// reference tests/wavelet.cc:88-113 (db8, periodic, 0..31)
TEST_CASE(wavelet_db8_golden) {
  float src[32], hi[16], lo[16];
  for (int i = 0; i < 32; i++) src[i] = i;
  wavelet_apply_na(WAVELET_TYPE_DAUBECHIES, 8, EXTENSION_TYPE_PERIODIC, src, 32, hi, lo);
  const float glo[16] = {1.4218407f, 4.2502678f, 7.0786950f, 9.9071221f, 12.735549f,
                         15.563976f, 18.392403f, 21.220831f, 24.049258f, 26.877685f,
                         29.706112f, 32.534539f, 35.362966f, 37.478254f, 45.304871f,
                         28.840594f};
  const float ghi_tail[3] = {-15.503000f, 5.5806650f, -1.3913732f};
  for (int i = 0; i < 16; i++) CHECK_NEAR(glo[i], lo[i], 5e-4);
  for (int i = 0; i < 13; i++) CHECK_NEAR(0.f, hi[i], 1e-4);
  for (int i = 0; i < 3; i++) CHECK_NEAR(ghi_tail[i], hi[13 + i], 5e-4);
  float *prep = wavelet_prepare_array(8, src, 32);
  float *h2 = wavelet_allocate_destination(8, 32), *l2 = wavelet_allocate_destination(8, 32);
  wavelet_apply(WAVELET_TYPE_DAUBECHIES, 8, EXTENSION_TYPE_PERIODIC, prep, 32, h2, l2);
  for (int i = 0; i < 16; i++) {
    CHECK_NEAR(hi[i], h2[i], 5e-4);
    CHECK_NEAR(lo[i], l2[i], 5e-4);
  }
  free(prep);
  free(h2);
  free(l2);
  CHECK_EQ(1, wavelet_validate_order(WAVELET_TYPE_DAUBECHIES, 8));
  CHECK_EQ(0, wavelet_validate_order(WAVELET_TYPE_COIFLET, 8));
}

// reference tests/detect_peaks.cc:43-75
TEST_CASE(detect_peaks_sin) {
  const int n = 4000;
  std::vector<float> x(n);
  for (int i = 0; i < n; i++) x[i] = std::sin(i * 3.14159265f / 100);
  for (int simd = 0; simd < 2; simd++) {
    ExtremumPoint *pts = nullptr;
    size_t count = 0;
    detect_peaks(simd, x.data(), n, kExtremumTypeBoth, &pts, &count);
    CHECK_EQ(40u, count);
    for (size_t i = 0; i < count; i++)
      CHECK_EQ(50 + 100 * static_cast<int>(i), pts[i].position);
    free(pts);
  }
}

// The vectorised host loops behind simd = 1 on host arrays (sum of lane-wise
// partial sums, lane-wise extremes, eight-position peak masks) at every
// length around their vector widths, on exact-size heap blocks so that an
// address sanitizer build sees any access past either end.
TEST_CASE(host_reductions_and_peaks_all_tails) {
  unsigned seed = 12345;
  auto next = [&seed] {
    seed = seed * 1664525u + 1013904223u;
    return static_cast<float>(static_cast<int>(seed >> 8) % 2001 - 1000) / 100.f;
  };
  for (size_t n = 1; n <= 100; n++) {
    float *x = static_cast<float *>(malloc(n * sizeof(float)));
    for (size_t i = 0; i < n; i++) x[i] = std::floor(next());  // equal neighbours happen
    double want = 0;
    float lo = x[0], hi = x[0];
    for (size_t i = 0; i < n; i++) {
      want += x[i];
      lo = std::min(lo, x[i]);
      hi = std::max(hi, x[i]);
    }
    CHECK_NEAR(want, static_cast<double>(sum_elements(x, n)), 1e-3);
    float mn = 0, mx = 0;
    minmax1D(1, x, static_cast<int>(n), &mn, &mx);
    CHECK_EQ(lo, mn);
    CHECK_EQ(hi, mx);
    if (n > 2) {
      for (int type = 1; type <= 3; type++) {
        ExtremumPoint *p0 = nullptr, *p1 = nullptr;
        size_t c0 = 0, c1 = 0;
        detect_peaks(0, x, n, static_cast<ExtremumType>(type), &p0, &c0);
        detect_peaks(1, x, n, static_cast<ExtremumType>(type), &p1, &c1);
        CHECK_EQ(c0, c1);
        for (size_t i = 0; i < c0 && i < c1; i++) {
          CHECK_EQ(p0[i].position, p1[i].position);
          CHECK_EQ(p0[i].value, p1[i].value);
        }
        free(p0);
        free(p1);
      }
    }
    free(x);
  }
}

// Host matrix products in 4 x 16 register blocks with zero-padded panels for
// the remainders: every tail combination on exact-size heap blocks.
TEST_CASE(host_matrix_multiply_all_tails) {
  unsigned seed = 99;
  auto next = [&seed] {
    seed = seed * 1664525u + 1013904223u;
    return static_cast<float>(static_cast<int>(seed >> 8) % 201 - 100) / 50.f;
  };
  for (size_t h1 = 1; h1 <= 9; h1++)
    for (size_t w2 : {1u, 15u, 16u, 17u, 31u, 32u, 40u})
      for (size_t w1 : {1u, 5u, 24u}) {
        float *a = static_cast<float *>(malloc(h1 * w1 * sizeof(float)));
        float *b = static_cast<float *>(malloc(w1 * w2 * sizeof(float)));
        float *bt = static_cast<float *>(malloc(w1 * w2 * sizeof(float)));
        float *r1 = static_cast<float *>(malloc(h1 * w2 * sizeof(float)));
        float *r0 = static_cast<float *>(malloc(h1 * w2 * sizeof(float)));
        for (size_t i = 0; i < h1 * w1; i++) a[i] = next();
        for (size_t i = 0; i < w1 * w2; i++) b[i] = next();
        for (size_t k = 0; k < w1; k++)
          for (size_t j = 0; j < w2; j++) bt[j * w1 + k] = b[k * w2 + j];
        matrix_multiply(0, a, b, w1, h1, w2, w1, r0);
        matrix_multiply(1, a, b, w1, h1, w2, w1, r1);
        for (size_t i = 0; i < h1 * w2; i++) CHECK_NEAR(r0[i], r1[i], 1e-4);
        matrix_multiply_transposed(1, a, bt, w1, h1, w1, w2, r1);
        for (size_t i = 0; i < h1 * w2; i++) CHECK_NEAR(r0[i], r1[i], 1e-4);
        free(a);
        free(b);
        free(bt);
        free(r1);
        free(r0);
      }
}

int main(int argc, char **argv) { return mini_test::run_all(argc, argv); }
