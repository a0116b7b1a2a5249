// wavelet.h (reference src/wavelet.c).  wavelet_apply / stationary_wavelet_
// apply run the HIP kernels of csrc/kernels/wavelet.hip; the *_na variants
// are the host reference.  The "prepared array" helpers keep the reference's
// non-AVX contract (the GPU needs no shifted copies).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/wavelet.h"

#include <cstdlib>
#include <cstring>

#include "csrc/api/dispatch.h"
#include "csrc/data/wavelet_tables.h"
#include "csrc/ref/ref.h"
#include "simd/gpu.h"
#include "simd/memory.h"

using vs::Staged;

namespace {
// The enum arguments come from C callers: their bits are read as an int and
// checked before anything uses them as the C++ enum (loading an
// out-of-range value through the enum type is undefined behaviour).
template <class E>
int enum_bits(const E &e) {
  static_assert(sizeof(E) == sizeof(int), "C enum representation");
  int v;
  std::memcpy(&v, &e, sizeof(v));
  return v;
}

#define VS_CHECK_DWT_ARGS(what) \
  check_dwt_args(what, enum_bits(type), order, enum_bits(ext), src, length, desthi, destlo)

void check_dwt_args(const char *what, int type, int order, int ext, const float *src,
                    size_t length, const float *hi, const float *lo) {
  if (!src || !hi || !lo) vs::fatal("%s: null pointer", what);
  if (type < WAVELET_TYPE_DAUBECHIES || type > WAVELET_TYPE_SYMLET ||
      !vs::wavelet_tables::valid(static_cast<WaveletType>(type), order))
    vs::fatal("%s: unsupported wavelet (type %d, order %d)", what, type, order);
  if (ext < EXTENSION_TYPE_PERIODIC || ext > EXTENSION_TYPE_ZERO)
    vs::fatal("%s: bad extension type %d", what, ext);
  if (length == 0) vs::fatal("%s: empty source", what);
}
}  // namespace

extern "C" {

int wavelet_validate_order(WaveletType type, int order) {
  return vs::wavelet_tables::valid(type, order) ? 1 : 0;
}

float *wavelet_prepare_array(int order, const float *src, size_t length) {
  (void)order;
  if (!src || length == 0 || length % 2) vs::fatal("wavelet_prepare_array: bad length");
  float *res = mallocf(length);
  if (res) std::memcpy(res, src, length * sizeof(float));
  return res;
}

float *wavelet_allocate_destination(int order, size_t sourceLength) {
  (void)order;
  if (sourceLength == 0 || sourceLength % 2)
    vs::fatal("wavelet_allocate_destination: bad length %zu", sourceLength);
  return mallocf(sourceLength / 2);
}

void wavelet_recycle_source(int order, float *src, size_t length,
                            float **desthihi, float **desthilo,
                            float **destlohi, float **destlolo) {
  (void)order;
  if (length == 0 || length % 4 != 0) {
    *desthihi = *desthilo = *destlohi = *destlolo = nullptr;
    return;
  }
  const size_t lq = length / 4;
  *desthihi = src;
  *desthilo = src + lq;
  *destlohi = src + lq * 2;
  *destlolo = src + lq * 3;
}

void wavelet_apply_na(WaveletType type, int order, ExtensionType ext,
                      const float *src, size_t length, float *desthi,
                      float *destlo) {
  VS_CHECK_DWT_ARGS("wavelet_apply_na");
  if (length % 2) vs::fatal("wavelet_apply_na: odd length %zu", length);
  vs::ref::dwt(type, order, ext, src, length, desthi, destlo);
}

void wavelet_apply(WaveletType type, int order, ExtensionType ext,
                   const float *src, size_t length, float *desthi,
                   float *destlo) {
  VS_CHECK_DWT_ARGS("wavelet_apply");
  if (length % 2) vs::fatal("wavelet_apply: odd length %zu", length);
  // Flag-less API (like arithmetic.h): GPU for device operands or enough
  // work per sample moved to amortise the host<->device round trip.
  if (!vs::api::use_gpu_wavelet(length, order, {src, desthi, destlo})) {
    vs::host::dwt(type, order, ext, src, length, desthi, destlo);
    return;
  }
  vs::api::run_sync("wavelet_apply", [&](hipStream_t s) {
    const size_t half = length / 2;
    Staged h(desthi, half * 4, Staged::kOut, s), l(destlo, half * 4, Staged::kOut, s);
    Staged x(src, length * 4, Staged::kIn, s);
    VS_TRY(h.status());
    VS_TRY(l.status());
    VS_TRY(x.status());
    VS_TRY(vs_dwt(type, order, ext, x.dev<float>(), static_cast<int64_t>(length), 0,
                  h.dev<float>(), l.dev<float>(), 0, 1, s));
    VS_TRY(h.finish());
    return l.finish();
  });
}

void stationary_wavelet_apply_na(WaveletType type, int order, int level,
                                 ExtensionType ext, const float *src,
                                 size_t length, float *desthi, float *destlo) {
  VS_CHECK_DWT_ARGS("stationary_wavelet_apply_na");
  if (level < 1) vs::fatal("stationary_wavelet_apply_na: level %d < 1", level);
  vs::ref::swt(type, order, level, ext, src, length, desthi, destlo);
}

void stationary_wavelet_apply(WaveletType type, int order, int level,
                              ExtensionType ext, const float *src,
                              size_t length, float *desthi, float *destlo) {
  VS_CHECK_DWT_ARGS("stationary_wavelet_apply");
  if (level < 1) vs::fatal("stationary_wavelet_apply: level %d < 1", level);
  if (!vs::api::use_gpu_wavelet(length, order, {src, desthi, destlo})) {
    vs::host::swt(type, order, level, ext, src, length, desthi, destlo);
    return;
  }
  vs::api::run_sync("stationary_wavelet_apply", [&](hipStream_t s) {
    Staged h(desthi, length * 4, Staged::kOut, s), l(destlo, length * 4, Staged::kOut, s);
    Staged x(src, length * 4, Staged::kIn, s);
    VS_TRY(h.status());
    VS_TRY(l.status());
    VS_TRY(x.status());
    VS_TRY(vs_swt(type, order, level, ext, x.dev<float>(), static_cast<int64_t>(length), 0,
                  h.dev<float>(), l.dev<float>(), 0, 1, s));
    VS_TRY(h.finish());
    return l.finish();
  });
}

}  // extern "C"
