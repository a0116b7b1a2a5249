// detect_peaks.h (reference src/detect_peaks.c:58-127).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/detect_peaks.h"

#include <cstdlib>
#include <vector>

#include "csrc/api/dispatch.h"
#include "csrc/ref/ref.h"
#include "simd/gpu.h"

using vs::Staged;

namespace {
constexpr size_t kSmallElems = 262144;  // noise (two of three samples an extremum): 108 us per 128 K on the host, 190 us through the GPU
}

extern "C" {

void detect_peaks(int simd, const float *data, size_t size, ExtremumType type,
                  ExtremumPoint **results, size_t *resultsLength) {
  if (!data || !results || !resultsLength || size <= 2)
    vs::fatal("detect_peaks: invalid arguments (size=%zu)", size);
  *results = nullptr;
  *resultsLength = 0;
  // short arrays stay on the host: two GPU round trips (count, then emit)
  // cost more than the two-pass host scan (about 1 ns per element)
  if (!simd) {
    vs::ref::detect_peaks(data, size, type, results, resultsLength);
    return;
  }
  if (!vs::api::use_gpu_simd(simd, "detect_peaks") ||
      vs::api::host_small(size, kSmallElems, {data})) {
    vs::host::detect_peaks(data, size, type, results, resultsLength);
    return;
  }
  unsigned long long total = 0;
  std::vector<int> pos;
  std::vector<float> val;
  vs::api::run_sync("detect_peaks", [&](hipStream_t s) {
    Staged x(data, size * 4, Staged::kIn, s);
    VS_TRY(x.status());
    vs::DeviceBuffer cnt;
    VS_TRY(cnt.alloc(sizeof(unsigned long long), s));
    // count first (one small read-back), then size the result exactly
    VS_TRY(vs_detect_peaks(x.dev<float>(), size, type, nullptr, nullptr, 0,
                           cnt.as<unsigned long long>(), s));
    VS_HIP(hipMemcpyAsync(&total, cnt.get(), sizeof(total), hipMemcpyDeviceToHost, s));
    VS_HIP(hipStreamSynchronize(s));
    if (total == 0) return VS_OK;
    vs::DeviceBuffer dpos, dval;
    VS_TRY(dpos.alloc(total * sizeof(int), s));
    VS_TRY(dval.alloc(total * sizeof(float), s));
    VS_TRY(vs_detect_peaks(x.dev<float>(), size, type, dpos.as<int>(), dval.as<float>(),
                           total, cnt.as<unsigned long long>(), s));
    pos.resize(total);
    val.resize(total);
    VS_HIP(hipMemcpyAsync(pos.data(), dpos.get(), total * sizeof(int),
                          hipMemcpyDeviceToHost, s));
    VS_HIP(hipMemcpyAsync(val.data(), dval.get(), total * sizeof(float),
                          hipMemcpyDeviceToHost, s));
    return VS_OK;
  });
  if (total == 0) return;
  auto *out = static_cast<ExtremumPoint *>(std::malloc(total * sizeof(ExtremumPoint)));
  for (size_t i = 0; i < total; i++) out[i] = ExtremumPoint{pos[i], val[i]};
  *results = out;
  *resultsLength = total;
}

}  // extern "C"
