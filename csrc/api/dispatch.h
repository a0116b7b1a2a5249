// Where does a host-API call run?  Shared policy of the source-compatible C
// API (the reference decides at compile time with #ifdef __AVX__ and at run
// time with the `int simd` flag, reference src/matrix.c:262-273).
//   * simd-flag functions: simd != 0 -> GPU (if one is present), 0 -> host
//     reference.  With no GPU the accelerated path degrades to the host
//     reference, as the reference does on a host without SIMD.
//   * flag-less array functions (arithmetic.h): GPU when an operand already
//     lives in device memory or the array has >= VELES_GPU_MIN_ELEMS elements.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#pragma once

#include <hip/hip_runtime_api.h>

#include <atomic>
#include <climits>
#include <cstddef>
#include <initializer_list>

#include "csrc/runtime/runtime.h"

namespace vs {
namespace api {

inline bool any_device(std::initializer_list<const void *> ptrs) {
  for (const void *p : ptrs)
    if (is_device_pointer(p)) return true;
  return false;
}

// The device API takes int dimensions: refuse, loudly, any size it cannot
// represent instead of truncating it (the reference API is size_t).
inline int checked_int(const char *what, size_t n) {
  if (n > static_cast<size_t>(INT_MAX))
    fatal("%s: size %zu exceeds the device path limit of %d", what, n, INT_MAX);
  return static_cast<int>(n);
}

inline bool use_gpu_simd(int simd, const char *fn) {
  if (!simd) return false;
  if (gpu_available()) return true;
  static std::atomic<bool> warned{false};  // calls may come from several threads
  if (!warned.exchange(true))
    log(1, "%s: no GPU visible, accelerated path runs the host reference", fn);
  return false;
}

// Limit for host_small() of calls that move more than they compute (sums and
// differences, conversions, normalisation): on pageable host operands the
// host loop is faster at every size, because the GPU path starts with a copy
// of every operand into pinned memory that costs as much as the loop itself
// (matrix_add 1024 x 1024: 100 us on the host, 480 us through the GPU).
constexpr size_t kHostAlways = size_t{1} << 44;

// simd != 0 calls on host operands whose work is below `limit` (elements or
// multiply-adds, scaled by VELES_HOST_SMALL_SCALE percent) run vectorised host
// loops: the GPU round trip alone costs 14-18 us.
inline bool host_small(size_t work, size_t limit, std::initializer_list<const void *> ptrs) {
  const size_t scale = host_small_scale();
  const bool below = limit >= kHostAlways ? scale != 0 : work < limit * scale / 100;
  return below && !any_device(ptrs);
}

// True when the GPU thresholds of the flag-less API are the explicit ones:
// VELES_GPU_MIN_ELEMS is set, or VELES_HOST_SMALL_SCALE is 0 (everything that
// can run on the GPU does; the test suite runs so).
inline bool explicit_gpu_threshold() {
  return gpu_min_elems_is_set() || host_small_scale() == 0;
}

// Flag-less streaming calls (arithmetic.h: conversions, products, sums): the
// GPU for device operands; for host operands only past an explicit threshold.
inline bool use_gpu_array(size_t n, std::initializer_list<const void *> ptrs) {
  if (!gpu_available()) return false;
  if (any_device(ptrs)) return true;
  return explicit_gpu_threshold() && n >= gpu_min_elems();
}

// One wavelet level on host operands: the host filter bank costs about
// 0.028 ns per sample and tap, the GPU path 20 us + 0.3 ns per sample (two
// pinned copies and the PCIe transfers), so the GPU pays from about
// length x (taps - 10) > 700,000 on (8 taps: never; 16 taps: 128 K samples;
// 76 taps: 11 K samples).
inline bool use_gpu_wavelet(size_t length, int order, std::initializer_list<const void *> ptrs) {
  if (!gpu_available()) return false;
  if (any_device(ptrs)) return true;
  if (explicit_gpu_threshold()) return length * static_cast<size_t>(order) >= gpu_min_elems();
  const size_t over = order > 10 ? static_cast<size_t>(order - 10) : 0;
  return length * over > 700000 * host_small_scale() / 100;
}

// Runs body(stream) on the library stream and waits for it; aborts with the
// library error message on failure (the host API has assert() semantics).
// Host operands go through one packed CallStaging per call (one H2D, one
// D2H, event polling; runtime.h).
template <class F>
void run_sync(const char *what, F &&body) {
  hipStream_t s = library_stream();
  CallStaging staging(s);
  vs_status st = body(s);
  if (st == VS_OK) st = staging.complete();
  if (st != VS_OK) fatal("%s: %s", what, last_error());
  log(2, "%s: done on GPU", what);
}

}  // namespace api
}  // namespace vs
