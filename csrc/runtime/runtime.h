// Runtime services shared by every API layer: device discovery, error
// reporting, stream-ordered scratch memory, host<->device staging, logging.
//
// The reference has no runtime (everything is a synchronous host call); this layer is what lets the source-compatible host API drive
// MI355X kernels: it decides where a call runs, stages host operands through
// the library's own non-blocking stream and synchronises before returning.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <cstdint>
#include <functional>
#include <string>
#include <vector>

#include "simd/gpu.h"

namespace vs {

// ---------------------------------------------------------------- errors
void set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();
const char *last_error();

// Returns VS_ERR_HIP (and records the message) if e != hipSuccess.
vs_status hip_status(hipError_t e, const char *what, const char *file,
                     int line);
#define VS_HIP(expr)                                                    \
  do {                                                                  \
    hipError_t vs_e_ = (expr);                                          \
    if (vs_e_ != hipSuccess)                                            \
      return ::vs::hip_status(vs_e_, #expr, __FILE__, __LINE__);        \
  } while (0)
#define VS_TRY(expr)                    \
  do {                                          \
    vs_status vs_s_ = (expr);                   \
    if (vs_s_ != VS_OK) return vs_s_;           \
  } while (0)
#define VS_REQUIRE(cond, ...)            \
  do {                                   \
    if (!(cond)) {                       \
      ::vs::set_error(__VA_ARGS__);      \
      return VS_ERR_INVALID;             \
    }                                    \
  } while (0)

// Aborts with a message; used by the void-returning reference-compatible
// host API, whose contract is assert() on misuse (e.g. src/matrix.c:300).
[[noreturn]] void fatal(const char *fmt, ...)
    __attribute__((format(printf, 1, 2)));
#define VS_CHECK_API(expr)                                              \
  do {                                                                  \
    vs_status vs_s_ = (expr);                                           \
    if (vs_s_ != VS_OK)                                                 \
      ::vs::fatal("%s failed: %s", #expr, ::vs::last_error());          \
  } while (0)

// ----------------------------------------------------------- batching
// Batched kernels put the batch on grid.y / grid.z (<= 65535 blocks); the
// public entry points walk larger batches in chunks of this size.
constexpr long long kMaxGridY = 65535;
template <class F>
vs_status batch_chunks(long long batch, F &&f) {
  for (long long b0 = 0; b0 < batch; b0 += kMaxGridY) {
    const long long nb = batch - b0 < kMaxGridY ? batch - b0 : kMaxGridY;
    VS_TRY(f(b0, static_cast<int>(nb)));
  }
  return VS_OK;
}

// --------------------------------------------------------------- logging
// VELES_LOG_LEVEL: 0 quiet (default), 1 dispatch decisions, 2 verbose.
int log_level();
void log(int level, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

// ---------------------------------------------------------------- device
bool gpu_available();
int device_count();
// Library stream of the current device (non-blocking, created lazily).
hipStream_t library_stream();
bool is_device_pointer(const void *p);
// Elements from which host-pointer array ops go to the GPU
// (VELES_GPU_MIN_ELEMS; 1 << 20 when unset, see api::explicit_gpu_threshold).
size_t gpu_min_elems();
bool gpu_min_elems_is_set();
// Percent applied to the small-call host limits of the simd = 1 host API
// (VELES_HOST_SMALL_SCALE, default 100; 0 sends every such call to the GPU).
size_t host_small_scale();
// Launch helper: grid size for a grid-stride elementwise kernel.
unsigned elementwise_grid(size_t work_items, unsigned block);
// Compute units of the current device (cached; 256 on MI355X), for sizing
// persistent grids.
int device_cu_count();

// ------------------------------------------------------- scratch memory
// Device scratch from the library's caching pool (stream-tagged blocks, see
// runtime.cpp); returned to the pool, stream-ordered, on destruction.
class DeviceBuffer {
 public:
  DeviceBuffer() = default;
  DeviceBuffer(size_t bytes, hipStream_t stream) { alloc(bytes, stream); }
  ~DeviceBuffer() { release(); }
  DeviceBuffer(const DeviceBuffer &) = delete;
  DeviceBuffer &operator=(const DeviceBuffer &) = delete;
  DeviceBuffer(DeviceBuffer &&o) noexcept { *this = std::move(o); }
  DeviceBuffer &operator=(DeviceBuffer &&o) noexcept {
    release();
    ptr_ = o.ptr_;
    bytes_ = o.bytes_;
    stream_ = o.stream_;
    o.ptr_ = nullptr;
    o.bytes_ = 0;
    return *this;
  }
  vs_status alloc(size_t bytes, hipStream_t stream);
  void release();
  template <class T>
  T *as() const {
    return static_cast<T *>(ptr_);
  }
  void *get() const { return ptr_; }
  size_t bytes() const { return bytes_; }

 private:
  void *ptr_ = nullptr;
  size_t bytes_ = 0;
  hipStream_t stream_ = nullptr;
};

// Frees every cached (unused) pool block.
void release_cached_memory();
// True when a DeviceBuffer of `bytes` would be refused because `stream` is
// being captured into a graph (scratch above 1 MiB per allocation is not
// taken inside a capture): callers with a scratch-free alternative use it.
bool scratch_refused_in_capture(size_t bytes, hipStream_t stream);

// ----------------------------------------------------------- staging
// Staging context of one host-API call (api::run_sync opens one per call).
// Host operands of up to 4 MiB (VELES_STAGE_MAX_KB) live in a pinned, device-mapped arena of the
// calling thread for the call: outputs and read-once inputs are accessed
// there by the kernels directly (zero-copy); inputs re-read by many
// workgroups (Staged::kReread) are packed and sent to a device arena with
// ONE host->device copy before the first kernel reads them (inputs of
// 128 KiB or more go at once, overlapping the packing of the next operand).  The call ends
// with one event wait and the copies to the caller's buffers.  Larger
// operands take the per-operand copy path; VELES_ZERO_COPY=0 moves every
// small operand to the device arena.
class CallStaging {
 public:
  explicit CallStaging(hipStream_t s);
  ~CallStaging();
  CallStaging(const CallStaging &) = delete;
  CallStaging &operator=(const CallStaging &) = delete;
  static CallStaging *current();
  // Reserves `bytes` in the arena (input: copied into the pinned image now);
  // returns the address kernels use (mapped host image when zero_copy, else
  // the device image), or nullptr (operand too large / arena full).
  void *reserve(const void *host_in, size_t bytes, bool zero_copy);
  // Issues the pending host->device copy of the re-read inputs.
  vs_status flush();
  // Output region [dev, dev + bytes) goes to `host` after the call.
  void add_output(void *dev, void *host, size_t bytes);
  // Event wait, then the outputs to the caller's buffers.
  vs_status complete();

 private:
  struct Out {
    size_t off, bytes;
    void *host;
    bool mapped;
  };
  hipStream_t stream_;
  CallStaging *prev_;
  size_t used_ = 0, pend_lo_ = 0, pend_hi_ = 0;
  std::vector<Out> outs_;
};

// Presents a host-or-device operand as a device pointer on `stream`.
// Device pointers pass through; host buffers are copied in (kIn), out on
// finish() (kOut) or both -- through the call's CallStaging when one is open.
class Staged {
 public:
  // kReread: an input that many workgroups read (convolution windows, GEMM
  // panels) -- staged into device memory, never read over the host link.
  enum Dir { kIn = 1, kOut = 2, kInOut = 3, kReread = 4, kInReread = 5 };
  Staged(const void *user, size_t bytes, Dir dir, hipStream_t stream);
  vs_status status() const { return status_; }
  template <class T>
  T *dev() const {
    // the packed copy of the call's inputs goes out before any kernel can
    // read this pointer
    if (packed_) (void)CallStaging::current()->flush();
    return static_cast<T *>(dev_);
  }
  // Copies device results back to the host buffer (kOut / kInOut).
  vs_status finish();

 private:
  void *user_;
  void *dev_ = nullptr;
  size_t bytes_;
  Dir dir_;
  hipStream_t stream_;
  DeviceBuffer buf_;
  vs_status status_ = VS_OK;
  bool packed_ = false;  // lives in the call's CallStaging arena
  bool pinned_ = false;  // pinned host operand on the DMA / in-place path
};

// Waits for everything queued on `s` so far by polling an event (lower
// latency than a blocking stream synchronise on a short call).
vs_status wait_stream(hipStream_t s);

// Element-wise maps over long pageable host arrays, in pieces through the two
// halves of the calling thread's pinned staging image: while the GPU works on
// one piece (reading and writing the image in place over the host link), the
// host copies the previous piece's results out and the next piece's inputs
// in.  A whole-array pass costs about 90 us per MiB (copy in, transfer and
// kernel, copy out, one after the other); the pieces overlap the three.
// The pieces' building blocks, for calls that are not plain maps (a long
// convolution cut into pieces with overlap-add): the calling thread's pinned
// staging image (host address, the GPU's view of the same pages, and a device
// buffer of the same size), one event per half, and the polling wait.
struct StageImage {
  char *host, *mapped, *dev;
  size_t bytes;
};
// False when pieces do not apply: staging switched to synchronous or device
// copies, VELES_PIPELINED_MAP=0, or no image.
bool stage_image(StageImage *out);
bool is_pageable_host(const void *p);
vs_status stage_half_event(int half, hipEvent_t *ev);
vs_status wait_event(hipEvent_t ev);

struct MapArray {
  const void *in;  // input array, or nullptr for an output
  void *out;       // output array, or nullptr for an input
  size_t elem;     // bytes per element
};
// launch(dev, count, stream) gets one device-visible pointer per array, in
// the order given, for `count` elements.
using MapLaunch = std::function<vs_status(void *const *dev, size_t count, hipStream_t s)>;
// False (and nothing done) when the pieces do not apply: an array in device
// or pinned memory, fewer than two pieces, staging switched to synchronous or
// device copies, or no image; the caller then takes the whole-array path.
bool pipelined_map(hipStream_t s, size_t n, const MapArray *arrays, int count,
                   const MapLaunch &launch, vs_status *status);

}  // namespace vs
