// Host paths for calls too small to be worth a GPU round trip (14-18 us on
// MI355X): direct convolution / correlation, single wavelet levels, small
// matrix sums and products.  The scalar functions of ref.cpp stay the
// semantic reference (simd = 0, `_na`); these compute the same sums with
// unit-stride inner loops the host compiler vectorises, built for the
// baseline ISA and for AVX2 + FMA and chosen at run time by CPU feature.
// The reference's counterparts are its hand-written AVX loops
// (reference src/convolve.c:49-100, src/wavelet.c:395-1555).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#include <immintrin.h>
#endif

#include "csrc/data/wavelet_tables.h"
#include "csrc/ref/ref.h"
#include "simd/gpu.h"

// Every loop body below is an always-inline function instantiated twice: for
// the baseline ISA and inside a function compiled for AVX2 + FMA, chosen once
// per process by CPU feature (`arch=` clones would match one CPU model only).
// (hipcc also parses this file for the device, where neither applies.)
#if defined(__x86_64__) && !defined(__HIP_DEVICE_COMPILE__)
#define VS_HOST_AVX2 1
#define VS_TARGET_AVX2 __attribute__((target("avx2,fma")))
#else
#define VS_HOST_AVX2 0
#define VS_TARGET_AVX2
#endif
#define VS_BODY static inline __attribute__((always_inline))

// multiply-adds of this file may fuse (the rest of the host code is built
// with contraction off to match the scalar reference bit for bit)
#pragma clang fp contract(fast)

namespace vs {
namespace host {
namespace {

// y[0 .. n) += a * x[0 .. n)
VS_BODY void axpy_body(float a, const float *__restrict__ x, float *__restrict__ y, long n) {
  for (long i = 0; i < n; i++) y[i] += a * x[i];
}

// y[n] = sum_m h[m] xp[n - m] for n in [0, ny), 64 outputs at a time held in
// registers over the whole tap loop: one load + one FMA per 8 products.
// xp points at x[0] inside a copy of x with 63 zeros before it and 63 after
// it (only taps that reach a real sample of the block are visited).
constexpr long kConvBlock = 64;
typedef float V8 __attribute__((vector_size(32)));
typedef float V8u __attribute__((vector_size(32), aligned(4)));
VS_BODY V8 splat8(float v) { return V8{v, v, v, v, v, v, v, v}; }
VS_BODY void conv_blocked_body(const float *__restrict__ xp, const float *__restrict__ h,
                              long nh, float *__restrict__ y, long ny) {
  const long nx = ny - nh + 1;
  for (long n0 = 0; n0 < ny; n0 += kConvBlock) {
    V8 a0 = {}, a1 = {}, a2 = {}, a3 = {}, a4 = {}, a5 = {}, a6 = {}, a7 = {};
    const float *p = xp + n0;
    // taps whose 64 samples are not all padding: n - m in [0, nx)
    const long m0 = std::max(0L, n0 - (nx - 1)), m1 = std::min(nh, n0 + kConvBlock);
    for (long m = m0; m < m1; m++) {
      const float hs = h[m];
      const V8 hm = {hs, hs, hs, hs, hs, hs, hs, hs};
      const V8u *q = reinterpret_cast<const V8u *>(p - m);
      a0 += hm * q[0];
      a1 += hm * q[1];
      a2 += hm * q[2];
      a3 += hm * q[3];
      a4 += hm * q[4];
      a5 += hm * q[5];
      a6 += hm * q[6];
      a7 += hm * q[7];
    }
    float acc[kConvBlock];
    V8u *o = reinterpret_cast<V8u *>(acc);
    o[0] = a0, o[1] = a1, o[2] = a2, o[3] = a3, o[4] = a4, o[5] = a5, o[6] = a6, o[7] = a7;
    const long w = std::min(kConvBlock, ny - n0);
    for (long j = 0; j < w; j++) y[n0 + j] = acc[j];
  }
}

// Two-channel filter bank over unit-stride runs: out[d] = sum_j c[j] run_j[d].
// The decimated level reads even / odd samples (tap j at offset j / 2 of ev
// or od), the stationary level one array (od = nullptr, tap j at offset
// j * stride).  16 outputs of both bands stay
// in registers over the tap loop.  The runs must be readable 15 floats past
// the last output.
VS_BODY void bank_body(const float *__restrict__ hp, const float *__restrict__ lp, int order,
                       const float *__restrict__ ev, const float *__restrict__ od,
                       long stride, float *__restrict__ hi, float *__restrict__ lo, long n) {
  for (long d0 = 0; d0 < n; d0 += 16) {
    V8 h0 = {}, h1 = {}, l0 = {}, l1 = {};
    for (int j = 0; j < order; j++) {
      const float *run = od ? ((j & 1) ? od : ev) + (j >> 1) + d0 : ev + j * stride + d0;
      const V8u *q = reinterpret_cast<const V8u *>(run);
      const float a = hp[j], b = lp[j];
      const V8 va = {a, a, a, a, a, a, a, a}, vb = {b, b, b, b, b, b, b, b};
      const V8 x0 = q[0], x1 = q[1];
      h0 += va * x0;
      h1 += va * x1;
      l0 += vb * x0;
      l1 += vb * x1;
    }
    if (d0 + 16 <= n) {
      V8u *oh = reinterpret_cast<V8u *>(hi + d0), *ol = reinterpret_cast<V8u *>(lo + d0);
      oh[0] = h0, oh[1] = h1, ol[0] = l0, ol[1] = l1;
    } else {
      float th[16], tl[16];
      V8u *oh = reinterpret_cast<V8u *>(th), *ol = reinterpret_cast<V8u *>(tl);
      oh[0] = h0, oh[1] = h1, ol[0] = l0, ol[1] = l1;
      for (long j = 0; d0 + j < n; j++) hi[d0 + j] = th[j], lo[d0 + j] = tl[j];
    }
  }
}

// Even and odd samples of src[0 .. 2 half) into ev / od.
VS_BODY void split_body(const float *__restrict__ src, long half, float *__restrict__ ev,
                        float *__restrict__ od) {
  for (long d = 0; d < half; d++) {
    ev[d] = src[2 * d];
    od[d] = src[2 * d + 1];
  }
}

// out[i] = a[i] + sign * b[i]
VS_BODY void addsub_body(const float *__restrict__ a, const float *__restrict__ b, float sign,
                         float *__restrict__ out, long n) {
  for (long i = 0; i < n; i++) out[i] = a[i] + sign * b[i];
}

// dot product with eight-lane partial sums
VS_BODY void dot_body(const float *__restrict__ a, const float *__restrict__ b, long n,
                      float *__restrict__ out) {
  V8 acc = {};
  long i = 0;
  for (; i + 8 <= n; i += 8)
    acc += *reinterpret_cast<const V8u *>(a + i) * *reinterpret_cast<const V8u *>(b + i);
  float r = ((acc[0] + acc[4]) + (acc[1] + acc[5])) + ((acc[2] + acc[6]) + (acc[3] + acc[7]));
  for (; i < n; i++) r += a[i] * b[i];
  *out = r;
}

// sum with 4 x 8 partial sums (the scalar loop is one dependent add per element)
VS_BODY void sum_body(const float *__restrict__ a, long n, float *__restrict__ out) {
  V8 s0 = {}, s1 = {}, s2 = {}, s3 = {};
  long i = 0;
  for (; i + 32 <= n; i += 32) {
    s0 += *reinterpret_cast<const V8u *>(a + i);
    s1 += *reinterpret_cast<const V8u *>(a + i + 8);
    s2 += *reinterpret_cast<const V8u *>(a + i + 16);
    s3 += *reinterpret_cast<const V8u *>(a + i + 24);
  }
  const V8 s = (s0 + s1) + (s2 + s3);
  float r = ((s[0] + s[4]) + (s[1] + s[5])) + ((s[2] + s[6]) + (s[3] + s[7]));
  for (; i < n; i++) r += a[i];
  *out = r;
}

// smallest and largest element; NaNs lose every comparison, as in the scalar loop
VS_BODY void minmax_body(const float *__restrict__ a, long n, float *__restrict__ out) {
  float lo = a[0], hi = a[0];
  long i = 0;
  if (n >= 16) {
    V8 l0, l1, h0, h1;
    for (int k = 0; k < 8; k++) l0[k] = l1[k] = h0[k] = h1[k] = a[0];
    for (; i + 16 <= n; i += 16) {
      const V8 u = *reinterpret_cast<const V8u *>(a + i);
      const V8 v = *reinterpret_cast<const V8u *>(a + i + 8);
      l0 = u < l0 ? u : l0;
      h0 = u > h0 ? u : h0;
      l1 = v < l1 ? v : l1;
      h1 = v > h1 ? v : h1;
    }
    for (int k = 0; k < 8; k++) {
      if (l0[k] < lo) lo = l0[k];
      if (l1[k] < lo) lo = l1[k];
      if (h0[k] > hi) hi = h0[k];
      if (h1[k] > hi) hi = h1[k];
    }
  }
  for (; i < n; i++) {
    if (a[i] < lo) lo = a[i];
    if (a[i] > hi) hi = a[i];
  }
  out[0] = lo;
  out[1] = hi;
}

// res[i][j] = sum_k a[i][k] b[k][j] for i in [0, rows) and j in [0, cols),
// rows a multiple of 4 and cols of 16: blocks of 4 x 16 results held in eight
// vector accumulators, so that each pair of b vectors loaded feeds eight
// multiply-adds (the row-by-row axpy form moves three vectors per one).
// b and res have row strides ldb and ldr.
VS_BODY void mm_block_body(const float *__restrict__ a, const float *__restrict__ b, long w1,
                           long ldb, long rows, long cols, float *__restrict__ res, long ldr) {
  for (long i = 0; i < rows; i += 4) {
    const float *a0 = a + i * w1, *a1 = a0 + w1, *a2 = a1 + w1, *a3 = a2 + w1;
    for (long j = 0; j < cols; j += 16) {
      V8 c00 = {}, c01 = {}, c10 = {}, c11 = {}, c20 = {}, c21 = {}, c30 = {}, c31 = {};
      const float *bp = b + j;
      for (long k = 0; k < w1; k++, bp += ldb) {
        const V8 b0 = *reinterpret_cast<const V8u *>(bp);
        const V8 b1 = *reinterpret_cast<const V8u *>(bp + 8);
        const V8 s0 = splat8(a0[k]), s1 = splat8(a1[k]), s2 = splat8(a2[k]), s3 = splat8(a3[k]);
        c00 += s0 * b0;
        c01 += s0 * b1;
        c10 += s1 * b0;
        c11 += s1 * b1;
        c20 += s2 * b0;
        c21 += s2 * b1;
        c30 += s3 * b0;
        c31 += s3 * b1;
      }
      float *r = res + i * ldr + j;
      *reinterpret_cast<V8u *>(r) = c00;
      *reinterpret_cast<V8u *>(r + 8) = c01;
      *reinterpret_cast<V8u *>(r + ldr) = c10;
      *reinterpret_cast<V8u *>(r + ldr + 8) = c11;
      *reinterpret_cast<V8u *>(r + 2 * ldr) = c20;
      *reinterpret_cast<V8u *>(r + 2 * ldr + 8) = c21;
      *reinterpret_cast<V8u *>(r + 3 * ldr) = c30;
      *reinterpret_cast<V8u *>(r + 3 * ldr + 8) = c31;
    }
  }
}

bool have_avx2() {
#if VS_HOST_AVX2
  static const bool yes = __builtin_cpu_supports("avx2") && __builtin_cpu_supports("fma");
  return yes;
#else
  return false;
#endif
}

#define VS_DISPATCH(name, params, args)                              \
  VS_TARGET_AVX2 void name##_avx2 params { name##_body args; }       \
  void name##_base params { name##_body args; }                      \
  inline void name params {                                          \
    if (have_avx2()) name##_avx2 args;                               \
    else name##_base args;                                           \
  }
VS_DISPATCH(axpy, (float a, const float *x, float *y, long n), (a, x, y, n))
VS_DISPATCH(conv_blocked, (const float *xp, const float *h, long nh, float *y, long ny),
            (xp, h, nh, y, ny))
VS_DISPATCH(bank, (const float *hp, const float *lp, int order, const float *ev,
                   const float *od, long stride, float *hi, float *lo, long n),
            (hp, lp, order, ev, od, stride, hi, lo, n))
VS_DISPATCH(split, (const float *src, long half, float *ev, float *od), (src, half, ev, od))
VS_DISPATCH(addsub, (const float *a, const float *b, float sign, float *out, long n),
            (a, b, sign, out, n))
VS_DISPATCH(dot, (const float *a, const float *b, long n, float *out), (a, b, n, out))
VS_DISPATCH(mm_block, (const float *a, const float *b, long w1, long ldb, long rows, long cols,
                       float *res, long ldr), (a, b, w1, ldb, rows, cols, res, ldr))
VS_DISPATCH(sum, (const float *a, long n, float *out), (a, n, out))
VS_DISPATCH(minmax, (const float *a, long n, float *out), (a, n, out))
#undef VS_DISPATCH

float extended(const float *src, long len, long idx, ExtensionType ext) {
  if (idx < len) return src[idx];
  const long t = idx - len;
  switch (ext) {
    case EXTENSION_TYPE_PERIODIC: return src[t % len];
    case EXTENSION_TYPE_MIRROR: return src[len - 1 - (t % len)];
    case EXTENSION_TYPE_CONSTANT: return src[len - 1];
    default: return 0.f;
  }
}

std::vector<float> &scratch(int which) {
  static thread_local std::vector<float> buf[2];
  return buf[which];
}

// Many taps: the axpy form moves three vectors per FMA; keep the outputs in
// registers instead.  The shorter operand plays the filter.
constexpr long kBlockedMinTaps = 24;
void blocked(const float *x, long nx, const float *h, long nh, bool reverse_h, float *y) {
  std::vector<float> &hr = scratch(1);
  if (reverse_h) {
    hr.resize(static_cast<size_t>(nh));
    std::reverse_copy(h, h + nh, hr.begin());
    h = hr.data();
  }
  if (nx < nh) {
    std::swap(x, h);
    std::swap(nx, nh);
  }
  std::vector<float> &xp = scratch(0);
  const long ny = nx + nh - 1;
  xp.resize(static_cast<size_t>(nx + 2 * kConvBlock));
  std::fill_n(xp.begin(), kConvBlock, 0.f);
  std::memcpy(xp.data() + kConvBlock, x, sizeof(float) * static_cast<size_t>(nx));
  std::fill_n(xp.begin() + kConvBlock + nx, kConvBlock, 0.f);
  conv_blocked(xp.data() + kConvBlock, h, nh, y, ny);
}

}  // namespace

// y[n] = sum_m h[m] x[n - m]: one pass of y[m ..] += h[m] * x per tap, taps
// in increasing order (the order ref::convolve_direct adds them in).
void convolve_direct(const float *x, size_t xl, const float *h, size_t hl, float *y) {
  const long nx = static_cast<long>(xl), nh = static_cast<long>(hl);
  if (std::min(nx, nh) >= kBlockedMinTaps) return blocked(x, nx, h, nh, false, y);
  std::memset(y, 0, sizeof(float) * static_cast<size_t>(nx + nh - 1));
  if (nx >= nh) {
    for (long m = 0; m < nh; m++) axpy(h[m], x, y + m, nx);
  } else {  // the longer operand in the inner loop
    for (long m = 0; m < nx; m++) axpy(x[m], h, y + m, nh);
  }
}

// r[k] = sum_m x[m] h[m + H - 1 - k]: the convolution with the reversed filter.
void correlate_direct(const float *x, size_t xl, const float *h, size_t hl, float *y) {
  const long nx = static_cast<long>(xl), nh = static_cast<long>(hl);
  if (std::min(nx, nh) >= kBlockedMinTaps) return blocked(x, nx, h, nh, true, y);
  std::memset(y, 0, sizeof(float) * static_cast<size_t>(nx + nh - 1));
  if (nx >= nh) {
    for (long m = 0; m < nh; m++) axpy(h[nh - 1 - m], x, y + m, nx);
  } else {
    std::vector<float> &hr = scratch(0);
    hr.resize(hl);
    std::reverse_copy(h, h + nh, hr.begin());
    for (long m = 0; m < nx; m++) axpy(x[m], hr.data(), y + m, nh);
  }
}

// One decimated level: the extended signal split into its even and odd
// samples, so tap j reads a unit-stride run of one of them.
void dwt(WaveletType type, int order, ExtensionType ext, const float *src, size_t len,
         float *hi, float *lo) {
  float hp[wavelet_tables::kMaxOrder], lp[wavelet_tables::kMaxOrder];
  wavelet_tables::make_filters(wavelet_tables::lowpass_f(type, order), order, hp, lp);
  const long n = static_cast<long>(len), half = n / 2;
  const long m = half + (order + 1) / 2;  // even / odd samples a level touches
  std::vector<float> &ev = scratch(0), &od = scratch(1);
  ev.resize(static_cast<size_t>(m + 16));
  od.resize(static_cast<size_t>(m + 16));
  split(src, half, ev.data(), od.data());
  for (long d = half; d < m; d++) {
    ev[d] = extended(src, n, 2 * d, ext);
    od[d] = extended(src, n, 2 * d + 1, ext);
  }
  bank(hp, lp, order, ev.data(), od.data(), 0, hi, lo, half);  // x~[2 d + j]
}

// One stationary level: tap r reads the extended signal at offset r 2^(level-1).
void swt(WaveletType type, int order, int level, ExtensionType ext, const float *src,
         size_t len, float *hi, float *lo) {
  float hp[wavelet_tables::kMaxOrder], lp[wavelet_tables::kMaxOrder];
  wavelet_tables::make_filters(wavelet_tables::lowpass_f(type, order), order, hp, lp);
  const long stride = 1L << (level - 1);
  const long n = static_cast<long>(len);
  const long m = n + (order - 1) * stride;
  std::vector<float> &xe = scratch(0);
  xe.resize(static_cast<size_t>(m + 16));
  std::memcpy(xe.data(), src, sizeof(float) * len);
  for (long i = n; i < m; i++) xe[i] = extended(src, n, i, ext);
  bank(hp, lp, order, xe.data(), nullptr, stride, hi, lo, n);
}

void matrix_add(const float *a, const float *b, size_t w, size_t h, float *res) {
  addsub(a, b, 1.f, res, static_cast<long>(w * h));
}

void matrix_sub(const float *a, const float *b, size_t w, size_t h, float *res) {
  addsub(a, b, -1.f, res, static_cast<long>(w * h));
}

#if VS_HOST_AVX2
}  // namespace host
}  // namespace vs
// glibc's vector math library (libmvec, shipped with glibc since 2.22): the
// AVX2 entry points of the x86-64 vector function ABI, eight lanes per call,
// at most 4 ulp off (measured here over the ranges of the tests: 1.9 ulp for
// sin / cos, 2.6 for exp, 3.9 for log near 1).
extern "C" {
VS_TARGET_AVX2 __m256 _ZGVdN8v_sinf(__m256);
VS_TARGET_AVX2 __m256 _ZGVdN8v_cosf(__m256);
VS_TARGET_AVX2 __m256 _ZGVdN8v_expf(__m256);
VS_TARGET_AVX2 __m256 _ZGVdN8v_logf(__m256);
VS_TARGET_AVX2 __m256 _ZGVdN8vv_powf(__m256, __m256);
}
namespace vs {
namespace host {
namespace {
VS_TARGET_AVX2 inline __m256 vfn(int fn, __m256 v, __m256 w) {
  switch (fn) {
    case VS_FN_SIN: return _ZGVdN8v_sinf(v);
    case VS_FN_COS: return _ZGVdN8v_cosf(v);
    case VS_FN_EXP: return _ZGVdN8v_expf(v);
    case VS_FN_LOG: return _ZGVdN8v_logf(v);
    case VS_FN_SQRT: return _mm256_sqrt_ps(v);
    default: return _ZGVdN8vv_powf(v, w);
  }
}

VS_TARGET_AVX2 void vmath_avx2(int fn, const float *x, const float *y, size_t n, float *res) {
  size_t i = 0;
  for (; i + 8 <= n; i += 8)
    _mm256_storeu_ps(res + i, vfn(fn, _mm256_loadu_ps(x + i),
                                  y ? _mm256_loadu_ps(y + i) : _mm256_setzero_ps()));
  if (i < n) {  // the last lanes through padded copies (1: inside every domain)
    alignas(32) float tx[8], ty[8], tr[8];
    for (size_t k = 0; k < 8; k++) {
      tx[k] = i + k < n ? x[i + k] : 1.f;
      ty[k] = y && i + k < n ? y[i + k] : 1.f;
    }
    _mm256_store_ps(tr, vfn(fn, _mm256_load_ps(tx), _mm256_load_ps(ty)));
    for (size_t k = 0; i + k < n; k++) res[i + k] = tr[k];
  }
}
}  // namespace
#endif

// res[i] = fn(x[i]) (fn: VS_FN_SIN ... VS_FN_SQRT of simd/gpu.h), or
// pow(x[i], y[i]) with y given; false when this CPU has no AVX2 (the caller
// then loops over libm).
bool vector_math(int fn, const float *x, const float *y, size_t n, float *res) {
#if VS_HOST_AVX2
  if (have_avx2()) {
    vmath_avx2(y ? -1 : fn, x, y, n, res);
    return true;
  }
#endif
  (void)fn, (void)x, (void)y, (void)n, (void)res;
  return false;
}

bool has_vector_math() { return have_avx2(); }

float sum_elements(const float *a, size_t n) {
  float r = 0.f;
  sum(a, static_cast<long>(n), &r);
  return r;
}

void minmax1d(const float *src, size_t n, float *mn, float *mx) {
  float out[2];
  minmax(src, static_cast<long>(n), out);
  if (mn) *mn = out[0];
  if (mx) *mx = out[1];
}

#if VS_HOST_AVX2
// Extrema of the kinds in `type` among x[1 .. n - 2], eight positions per
// step: the tests of the scalar loop as lane masks, one bit per position.
// With pts == nullptr the extrema are only counted.
VS_TARGET_AVX2 long peaks_avx2(const float *x, long n, int type, ExtremumPoint *pts) {
  const __m256 zero = _mm256_setzero_ps();
  const __m256 want_max = _mm256_castsi256_ps(
      _mm256_set1_epi32((type & kExtremumTypeMaximum) ? -1 : 0));
  const __m256 want_min = _mm256_castsi256_ps(
      _mm256_set1_epi32((type & kExtremumTypeMinimum) ? -1 : 0));
  long k = 0, i = 1;
  for (; i + 8 < n; i += 8) {
    const __m256 c = _mm256_loadu_ps(x + i);
    const __m256 d1 = _mm256_sub_ps(c, _mm256_loadu_ps(x + i - 1));
    const __m256 d2 = _mm256_sub_ps(c, _mm256_loadu_ps(x + i + 1));
    const __m256 ext = _mm256_cmp_ps(_mm256_mul_ps(d1, d2), zero, _CMP_GT_OQ);
    const __m256 kind = _mm256_or_ps(
        _mm256_and_ps(_mm256_cmp_ps(d1, zero, _CMP_GT_OQ), want_max),
        _mm256_and_ps(_mm256_cmp_ps(d1, zero, _CMP_LT_OQ), want_min));
    unsigned m = static_cast<unsigned>(_mm256_movemask_ps(_mm256_and_ps(ext, kind)));
    if (!pts) {
      k += __builtin_popcount(m);
      continue;
    }
    while (m) {
      const long p = i + __builtin_ctz(m);
      pts[k++] = ExtremumPoint{static_cast<int>(p), x[p]};
      m &= m - 1;
    }
  }
  for (; i + 1 < n; i++) {
    const float d1 = x[i] - x[i - 1], d2 = x[i] - x[i + 1];
    if (d1 * d2 > 0 && ((d1 > 0 && (type & kExtremumTypeMaximum)) ||
                        (d1 < 0 && (type & kExtremumTypeMinimum)))) {
      if (pts) pts[k] = ExtremumPoint{static_cast<int>(i), x[i]};
      k++;
    }
  }
  return k;
}
#endif

// Two passes, count then write, so that the result is allocated once at its
// final size and no pass branches on the data.
void detect_peaks(const float *x, size_t n, ExtremumType type, ExtremumPoint **out,
                  size_t *count) {
#if VS_HOST_AVX2
  if (have_avx2()) {
    const long c = peaks_avx2(x, static_cast<long>(n), static_cast<int>(type), nullptr);
    *count = static_cast<size_t>(c);
    *out = nullptr;
    if (c == 0) return;
    auto *pts = static_cast<ExtremumPoint *>(
        std::malloc(static_cast<size_t>(c) * sizeof(ExtremumPoint)));
    if (!pts) {
      *count = 0;
      return;
    }
    peaks_avx2(x, static_cast<long>(n), static_cast<int>(type), pts);
    *out = pts;
    return;
  }
#endif
  ref::detect_peaks(x, n, type, out, count);
}

// res (h1 x w2) = a (h1 x w1) b (w1 x w2): row i of res accumulates
// a[i][k] * (row k of b), unit stride over w2.
void matrix_multiply(const float *a, const float *b, size_t w1, size_t h1, size_t w2,
                     float *res) {
  const long W1 = static_cast<long>(w1), W2 = static_cast<long>(w2);
  const long rows = static_cast<long>(h1 & ~size_t{3}), cols = static_cast<long>(w2 & ~size_t{15});
  const long rem_r = static_cast<long>(h1) - rows, rem_c = W2 - cols;
  if (rows && cols) mm_block(a, b, W1, W2, rows, cols, res, W2);
  // The last h1 % 4 rows and w2 % 16 columns go through the same blocks on
  // zero-padded copies: the rows of a in a 4 x w1 panel, the columns of b in
  // a w1 x 16 panel, results in a 4-row or 16-column buffer.
  std::vector<float> &pa = scratch(0), &pb = scratch(1);
  static thread_local std::vector<float> out;
  if (rem_r) {
    pa.assign(static_cast<size_t>(4 * W1), 0.f);
    std::memcpy(pa.data(), a + rows * W1, sizeof(float) * static_cast<size_t>(rem_r * W1));
  }
  if (rem_c) {
    pb.assign(static_cast<size_t>(16 * W1), 0.f);
    for (long k = 0; k < W1; k++)
      std::memcpy(pb.data() + 16 * k, b + k * W2 + cols, sizeof(float) * static_cast<size_t>(rem_c));
  }
  if (rem_c && rows) {  // right strip
    out.resize(static_cast<size_t>(rows * 16));
    mm_block(a, pb.data(), W1, 16, rows, 16, out.data(), 16);
    for (long i = 0; i < rows; i++)
      std::memcpy(res + i * W2 + cols, out.data() + 16 * i, sizeof(float) * static_cast<size_t>(rem_c));
  }
  if (rem_r && cols) {  // bottom strip
    out.resize(static_cast<size_t>(4 * cols));
    mm_block(pa.data(), b, W1, W2, 4, cols, out.data(), cols);
    for (long i = 0; i < rem_r; i++)
      std::memcpy(res + (rows + i) * W2, out.data() + i * cols, sizeof(float) * static_cast<size_t>(cols));
  }
  if (rem_r && rem_c) {  // corner
    out.resize(64);
    mm_block(pa.data(), pb.data(), W1, 16, 4, 16, out.data(), 16);
    for (long i = 0; i < rem_r; i++)
      std::memcpy(res + (rows + i) * W2 + cols, out.data() + 16 * i,
                  sizeof(float) * static_cast<size_t>(rem_c));
  }
}

// res (h1 x h2) = a (h1 x w1) b^T, b stored h2 x w1: row-by-row dot products.
void matrix_multiply_transposed(const float *a, const float *b, size_t w1, size_t h1,
                                size_t h2, float *res) {
  if (h1 >= 8 && h2 >= 16) {  // enough rows to pay for transposing b once
    static thread_local std::vector<float> bt;  // matrix_multiply uses the shared scratch
    bt.resize(w1 * h2);
    for (size_t j = 0; j < h2; j++)
      for (size_t k = 0; k < w1; k++) bt[k * h2 + j] = b[j * w1 + k];
    matrix_multiply(a, bt.data(), w1, h1, h2, res);
    return;
  }
  for (size_t i = 0; i < h1; i++)
    for (size_t j = 0; j < h2; j++)
      dot(a + i * w1, b + j * w1, static_cast<long>(w1), res + i * h2 + j);
}

}  // namespace host
}  // namespace vs
