// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "csrc/ref/ref.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "csrc/data/wavelet_tables.h"

namespace vs {
namespace ref {

void matrix_add(const float *a, const float *b, size_t w, size_t h,
                float *res) {
  const size_t n = w * h;
  for (size_t i = 0; i < n; i++) res[i] = a[i] + b[i];
}

void matrix_sub(const float *a, const float *b, size_t w, size_t h,
                float *res) {
  const size_t n = w * h;
  for (size_t i = 0; i < n; i++) res[i] = a[i] - b[i];
}

void matrix_multiply(const float *a, const float *b, size_t w1, size_t h1,
                     size_t w2, float *res) {
  // i-k-j order: same products and the same k-ordered fp32 sums per output
  // as the reference's i-j-k loop, cache friendly.
  std::vector<float> row(w2);
  for (size_t i = 0; i < h1; i++) {
    std::fill(row.begin(), row.end(), 0.f);
    for (size_t k = 0; k < w1; k++) {
      const float av = a[i * w1 + k];
      const float *brow = b + k * w2;
      for (size_t j = 0; j < w2; j++) row[j] += av * brow[j];
    }
    std::copy(row.begin(), row.end(), res + i * w2);
  }
}

void matrix_multiply_transposed(const float *a, const float *b, size_t w1,
                                size_t h1, size_t h2, float *res) {
  for (size_t i = 0; i < h1; i++) {
    for (size_t j = 0; j < h2; j++) {
      float s = 0.f;
      for (size_t k = 0; k < w1; k++) s += a[i * w1 + k] * b[j * w1 + k];
      res[i * h2 + j] = s;
    }
  }
}

void convolve_direct(const float *x, size_t xl, const float *h, size_t hl,
                     float *y) {
  const long nx = static_cast<long>(xl), nh = static_cast<long>(hl);
  for (long n = 0; n < nx + nh - 1; n++) {
    const long beg = n < nx ? 0 : n - nx + 1;
    const long end = std::min(n + 1, nh);
    float s = 0.f;
    for (long m = beg; m < end; m++) s += h[m] * x[n - m];
    y[n] = s;
  }
}

void correlate_direct(const float *x, size_t xl, const float *h, size_t hl,
                      float *y) {
  // r[k] = sum_m x[m] h[m + H - 1 - k]   (reference src/correlate.c:78-125)
  const long nx = static_cast<long>(xl), nh = static_cast<long>(hl);
  for (long n = nh - 1; n > -nx; n--) {
    const long beg = n <= 0 ? -n : 0;
    const long end = std::min(-n + nh, nx);
    float s = 0.f;
    for (long m = beg; m < end; m++) s += x[m] * h[n + m];
    y[-n + nh - 1] = s;
  }
}

void fft_inplace(double *d, size_t n, bool inverse) {
  // bit reversal
  for (size_t i = 1, j = 0; i < n; i++) {
    size_t bit = n >> 1;
    for (; j & bit; bit >>= 1) j ^= bit;
    j ^= bit;
    if (i < j) {
      std::swap(d[2 * i], d[2 * j]);
      std::swap(d[2 * i + 1], d[2 * j + 1]);
    }
  }
  const double sign = inverse ? 1.0 : -1.0;
  for (size_t len = 2; len <= n; len <<= 1) {
    const double ang = sign * 2.0 * M_PI / static_cast<double>(len);
    for (size_t i = 0; i < n; i += len) {
      for (size_t k = 0; k < len / 2; k++) {
        const double wr = std::cos(ang * k), wi = std::sin(ang * k);
        double *u = d + 2 * (i + k), *v = d + 2 * (i + k + len / 2);
        const double tr = v[0] * wr - v[1] * wi;
        const double ti = v[0] * wi + v[1] * wr;
        v[0] = u[0] - tr;
        v[1] = u[1] - ti;
        u[0] += tr;
        u[1] += ti;
      }
    }
  }
}

void convolve_fft(const float *x, size_t xl, const float *h, size_t hl,
                  int reverse_h, float *y) {
  const size_t out = xl + hl - 1;
  size_t m = 1;
  while (m < out) m <<= 1;
  // x in the real part, h in the imaginary part: one complex FFT gives both
  // spectra (X[k] = (Z[k] + conj Z[m-k]) / 2, H[k] = (Z[k] - conj Z[m-k])/2i).
  std::vector<double> z(2 * m, 0.0);
  for (size_t i = 0; i < xl; i++) z[2 * i] = x[i];
  for (size_t i = 0; i < hl; i++)
    z[2 * i + 1] = reverse_h ? h[hl - 1 - i] : h[i];
  fft_inplace(z.data(), m, false);
  std::vector<double> p(2 * m);
  for (size_t k = 0; k < m; k++) {
    const size_t q = (m - k) % m;
    const double ar = z[2 * k], ai = z[2 * k + 1];
    const double br = z[2 * q], bi = -z[2 * q + 1];
    const double xr = 0.5 * (ar + br), xi = 0.5 * (ai + bi);
    const double hr = 0.5 * (ai - bi), hi = -0.5 * (ar - br);
    p[2 * k] = xr * hr - xi * hi;
    p[2 * k + 1] = xr * hi + xi * hr;
  }
  fft_inplace(p.data(), m, true);
  for (size_t i = 0; i < out; i++)
    y[i] = static_cast<float>(p[2 * i] / static_cast<double>(m));
}

void minmax2d(const uint8_t *src, int stride, int w, int h, uint8_t *mn,
              uint8_t *mx) {
  uint8_t lo = src[0], hi = src[0];
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const uint8_t v = src[y * stride + x];
      lo = std::min(lo, v);
      hi = std::max(hi, v);
    }
  if (mn) *mn = lo;
  if (mx) *mx = hi;
}

void normalize2d_minmax(uint8_t mn, uint8_t mx, const uint8_t *src,
                        int sstride, int w, int h, float *dst, int dstride) {
  if (mx == mn) {
    for (int y = 0; y < h; y++)
      for (int x = 0; x < w; x++) dst[y * dstride + x] = 0.f;
    return;
  }
  const float diff = (mx - mn) / 2.f;
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++)
      dst[y * dstride + x] = (src[y * sstride + x] - mn) / diff - 1.0f;
}

void minmax1d(const float *src, int n, float *mn, float *mx) {
  float lo = src[0], hi = src[0];
  for (int i = 0; i < n; i++) {
    const float v = src[i];
    if (v < lo) lo = v;
    if (v > hi) hi = v;
  }
  if (mn) *mn = lo;
  if (mx) *mx = hi;
}

void detect_peaks(const float *x, size_t n, ExtremumType type,
                  ExtremumPoint **out, size_t *count) {
  std::vector<ExtremumPoint> pts;
  for (size_t i = 1; i + 1 < n; i++) {
    const float d1 = x[i] - x[i - 1];
    const float d2 = x[i] - x[i + 1];
    if (d1 * d2 > 0) {
      if ((d1 > 0 && (type & kExtremumTypeMaximum)) ||
          (d1 < 0 && (type & kExtremumTypeMinimum)))
        pts.push_back(ExtremumPoint{static_cast<int>(i), x[i]});
    }
  }
  *count = pts.size();
  *out = nullptr;
  if (!pts.empty()) {
    *out = static_cast<ExtremumPoint *>(
        std::malloc(pts.size() * sizeof(ExtremumPoint)));
    std::copy(pts.begin(), pts.end(), *out);
  }
}

namespace {
// Sample idx of the signal extended past its end (reference
// src/wavelet.c:248-269: ext[t] for t = idx - len).
inline float extended(const float *src, long len, long idx,
                      ExtensionType ext) {
  if (idx < len) return src[idx];
  const long t = idx - len;
  switch (ext) {
    case EXTENSION_TYPE_PERIODIC:
      return src[t % len];
    case EXTENSION_TYPE_MIRROR:
      return src[len - 1 - (t % len)];
    case EXTENSION_TYPE_CONSTANT:
      return src[len - 1];
    case EXTENSION_TYPE_ZERO:
    default:
      return 0.f;
  }
}
}  // namespace

void dwt(WaveletType type, int order, ExtensionType ext, const float *src,
         size_t len, float *hi, float *lo) {
  float hp[wavelet_tables::kMaxOrder], lp[wavelet_tables::kMaxOrder];
  wavelet_tables::make_filters(wavelet_tables::lowpass_f(type, order), order,
                               hp, lp);
  const long n = static_cast<long>(len);
  for (long i = 0, d = 0; i < n; i += 2, d++) {
    float sh = 0.f, sl = 0.f;
    for (int j = 0; j < order; j++) {
      const float v = extended(src, n, i + j, ext);
      sh += hp[j] * v;
      sl += lp[j] * v;
    }
    hi[d] = sh;
    lo[d] = sl;
  }
}

void swt(WaveletType type, int order, int level, ExtensionType ext,
         const float *src, size_t len, float *hi, float *lo) {
  float hp[wavelet_tables::kMaxOrder], lp[wavelet_tables::kMaxOrder];
  wavelet_tables::make_filters(wavelet_tables::lowpass_f(type, order), order,
                               hp, lp);
  const long stride = 1L << (level - 1);
  const long n = static_cast<long>(len);
  for (long i = 0; i < n; i++) {
    float sh = 0.f, sl = 0.f;
    for (int r = 0; r < order; r++) {
      const float v = extended(src, n, i + r * stride, ext);
      sh += hp[r] * v;
      sl += lp[r] * v;
    }
    hi[i] = sh;
    lo[i] = sl;
  }
}

}  // namespace ref
}  // namespace vs
