// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "csrc/runtime/runtime.h"

#include <unistd.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <chrono>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <vector>

namespace vs {

namespace {
thread_local std::string g_error;

int env_int(const char *name, int dflt) {
  const char *v = std::getenv(name);
  if (!v || !*v) return dflt;
  return std::atoi(v);
}
}  // namespace

void set_error(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_error = buf;
  log(2, "error: %s", buf);
}

void clear_error() { g_error.clear(); }
const char *last_error() { return g_error.c_str(); }

vs_status hip_status(hipError_t e, const char *what, const char *file,
                     int line) {
  set_error("%s: %s (%s:%d)", what, hipGetErrorString(e), file, line);
  return VS_ERR_HIP;
}

void fatal(const char *fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::fprintf(stderr, "veles.simd: fatal: %s\n", buf);
  std::fflush(stderr);
  std::abort();
}

int log_level() {
  static const int level = env_int("VELES_LOG_LEVEL", 0);
  return level;
}

void log(int level, const char *fmt, ...) {
  if (level > log_level()) return;
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  std::fprintf(stderr, "[veles.simd] %s\n", buf);
}

int device_count() {
  static const int count = [] {
    if (env_int("VELES_DISABLE_GPU", 0)) return 0;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
      (void)hipGetLastError();
      n = 0;
    }
    return n;
  }();
  return count;
}

bool gpu_available() { return device_count() > 0; }

hipStream_t library_stream() {
  static std::mutex mu;
  static std::vector<hipStream_t> streams;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lock(mu);
  if (streams.size() <= static_cast<size_t>(dev))
    streams.resize(dev + 1, nullptr);
  if (!streams[dev]) {
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
      fatal("cannot create the library stream on device %d", dev);
    streams[dev] = s;
  }
  return streams[dev];
}

// The program break heap [start_brk, sbrk(0)) belongs to malloc: no device or
// pinned allocation can live there, so small malloc'd operands (the tiny host
// calls, where three hipPointerGetAttributes queries of ~0.1 us each would
// cost more than the work) are classified without asking the HIP runtime.
static bool in_brk_heap(const void *p) {
  static const uintptr_t start = [] {
    // field 47 of /proc/self/stat (after the parenthesised command name)
    uintptr_t v = 0;
    if (FILE *f = std::fopen("/proc/self/stat", "r")) {
      char buf[2048];
      const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
      std::fclose(f);
      buf[n] = 0;
      if (const char *q = std::strrchr(buf, ')')) {
        int field = 2;
        for (q++; *q && field < 47; q++)
          if (*q == ' ') field++;
        if (field == 47) v = static_cast<uintptr_t>(std::strtoull(q, nullptr, 10));
      }
    }
    return v;
  }();
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  return start && a >= start && a < reinterpret_cast<uintptr_t>(sbrk(0));
}

bool is_device_pointer(const void *p) {
  if (!p || !gpu_available() || in_brk_heap(p)) return false;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeDevice ||
         attr.type == hipMemoryTypeManaged;
}

size_t gpu_min_elems() {
  static const size_t n = [] {
    const char *v = std::getenv("VELES_GPU_MIN_ELEMS");
    if (!v || !*v) return static_cast<size_t>(1) << 20;
    return static_cast<size_t>(std::strtoull(v, nullptr, 10));
  }();
  return n;
}

bool gpu_min_elems_is_set() {
  static const bool set = [] {
    const char *v = std::getenv("VELES_GPU_MIN_ELEMS");
    return v && *v;
  }();
  return set;
}

size_t host_small_scale() {
  static const size_t n = [] {
    const char *v = std::getenv("VELES_HOST_SMALL_SCALE");
    if (!v || !*v) return static_cast<size_t>(100);
    return static_cast<size_t>(std::strtoull(v, nullptr, 10));
  }();
  return n;
}

unsigned elementwise_grid(size_t work_items, unsigned block) {
  // One work item per thread up to 2^20 blocks (2^28 threads), grid-stride
  // beyond.  Measured on 2^26-element fp32 maps: a 2048-block grid-stride
  // grid reaches 5.0-5.6 TB/s, one item per thread 5.9-6.2 TB/s
  // (profiles/r1/session5/elementwise_grid_cap_ab.md).  VS_EW_GRID_CAP
  // overrides the cap for tuning runs.
  static const size_t cap = [block] {
    // HIP limits gridDim.x * blockDim.x to < 2^32 threads.
    const size_t hw_max = (size_t{0xffffffffu}) / (block ? block : 256);
    const char *e = std::getenv("VS_EW_GRID_CAP");
    if (!e) return size_t{1} << 20;
    char *end = nullptr;
    const unsigned long long v = std::strtoull(e, &end, 10);
    if (end == e || *end != '\0' || v == 0) {
      std::fprintf(stderr, "veles.simd: ignoring VS_EW_GRID_CAP=%s (not a positive integer)\n", e);
      return size_t{1} << 20;
    }
    if (v > hw_max) {
      std::fprintf(stderr, "veles.simd: VS_EW_GRID_CAP=%llu clamped to %zu\n", v, hw_max);
      return hw_max;
    }
    return static_cast<size_t>(v);
  }();
  size_t g = (work_items + block - 1) / block;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  return static_cast<unsigned>(g);
}

int device_cu_count() {
  static int cache[64] = {};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  if (cache[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0) {
      (void)hipGetLastError();
      n = 256;
    }
    cache[dev] = n;
  }
  return cache[dev];
}

static bool sync_stage() {
  static const bool v = env_int("VELES_SYNC_STAGE", 0) != 0;
  return v;
}

// Caching device allocator for library scratch and host staging.  Blocks are
// tagged with the stream that released them and are reused by that stream
// only (stream order makes immediate reuse safe); other streams allocate
// their own.  Nothing is recorded at release: an event record between two
// kernels of a call sequence put a ~6 us gap into the queue (rocprofv3 trace
// of the conv filter / block kernels, profiles/r2/conv/alloc_gap.md), and
// the stream handle is only compared, never passed to the runtime, so a
// stream the caller has since destroyed is harmless -- provided no new
// stream is handed the destroyed stream's handle while work of the old one
// that uses a cached block is still queued (hipStreamDestroy returns before
// that work ends): a host that destroys streams with library calls still in
// flight must synchronise them first.  The out-of-memory purge synchronises
// the device before freeing, and so does the trim that keeps the cached
// bytes under VELES_SCRATCH_CACHE_MB.  (The HIP
// stream-ordered pool -- hipMallocAsync -- returned stale results on ROCm 7.2
// after block reuse in our C API tests; this pool avoids depending on it.)
class ScratchPool {
 public:
  static ScratchPool &get() {
    static ScratchPool *pool = new ScratchPool();  // never destroyed
    return *pool;
  }

  void *alloc(size_t bytes, hipStream_t stream) {
    const size_t sz = round(bytes);
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (capturing(stream)) {
      // Inside a HIP-graph capture: a stream-ordered allocation becomes a
      // graph memory node owned by the graph (freed by the matching
      // hipFreeAsync node); the cache (event queries, host-side reuse) is
      // not usable while capturing.
      // Only small scratch is taken this way.  A captured pipeline whose
      // scratch ran to several MiB per allocation (partitioned overlap-save
      // spectra, tiled pyramid bands) faulted the GPU when the graph was
      // replayed; captures of pipelines with allocations up to tens of KiB
      // replay correctly (tests/test_graphs.py).  Larger requests are refused
      // so such a pipeline fails at capture with an error instead.
      if (sz > kCaptureAllocMax) return nullptr;
      void *p = nullptr;
      if (hipMallocAsync(&p, sz, stream) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
      }
      std::lock_guard<std::mutex> lock(mu_);
      graph_.insert(p);
      return p;
    }
    {
      std::lock_guard<std::mutex> lock(mu_);
      for (auto it = free_.lower_bound(sz); it != free_.end(); ++it) {
        if (it->first > 2 * sz + (1 << 20)) break;  // too wasteful
        Block &b = it->second;
        if (b.device != dev) continue;
        if (b.stream != stream) continue;
        void *p = b.ptr;
        live_[p] = b;
        cached_ -= b.size;
        free_.erase(it);
        return p;
      }
    }
    void *p = nullptr;
    if (hipMalloc(&p, sz) != hipSuccess) {
      (void)hipGetLastError();
      release_all_free();  // retry once after dropping the cache
      if (hipMalloc(&p, sz) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
      }
    }
    std::lock_guard<std::mutex> lock(mu_);
    live_[p] = Block{p, sz, dev, stream, 0};
    return p;
  }

  void release(void *p, hipStream_t stream) {
    std::lock_guard<std::mutex> lock(mu_);
    if (graph_.erase(p)) {
      (void)hipFreeAsync(p, stream);
      return;
    }
    auto it = live_.find(p);
    if (it == live_.end()) return;
    Block b = it->second;
    live_.erase(it);
    b.stream = stream;
    b.tick = ++tick_;
    free_.emplace(b.size, b);
    cached_ += b.size;
    if (cached_ > cap_bytes()) trim_locked();
  }

  // Cached bytes above the cap (a host that cycles through many streams
  // builds one cache per stream): synchronise once, then free the blocks
  // released longest ago until half the cap is left.
  void trim_locked() {
    (void)hipDeviceSynchronize();
    std::vector<std::multimap<size_t, Block>::iterator> order;
    for (auto it = free_.begin(); it != free_.end(); ++it) order.push_back(it);
    std::sort(order.begin(), order.end(),
              [](const auto &a, const auto &b) { return a->second.tick < b->second.tick; });
    for (auto it : order) {
      if (cached_ <= cap_bytes() / 2) break;
      cached_ -= it->second.size;
      (void)hipFree(it->second.ptr);
      free_.erase(it);
    }
  }

  static size_t cap_bytes() {
    static const size_t v = static_cast<size_t>(env_int("VELES_SCRATCH_CACHE_MB", 8192)) << 20;
    return v;
  }

  size_t cached_bytes() {
    std::lock_guard<std::mutex> lock(mu_);
    return cached_;
  }

  // True when alloc() refuses `bytes` because `stream` is being captured.
  static bool refused_in_capture(size_t bytes, hipStream_t stream) {
    return round(bytes) > kCaptureAllocMax && capturing(stream);
  }

  void release_all_free() {
    std::lock_guard<std::mutex> lock(mu_);
    if (!free_.empty()) (void)hipDeviceSynchronize();
    for (auto &kv : free_) (void)hipFree(kv.second.ptr);
    free_.clear();
    cached_ = 0;
  }

 private:
  struct Block {
    void *ptr;
    size_t size;
    int device;
    hipStream_t stream;
    uint64_t tick = 0;  // release order (trim_locked frees the oldest first)
  };
  static size_t round(size_t b) {
    if (b <= (1u << 20)) {
      size_t s = 512;
      while (s < b) s <<= 1;
      return s;
    }
    const size_t g = 2u << 20;
    return (b + g - 1) / g * g;
  }
  static constexpr size_t kCaptureAllocMax = static_cast<size_t>(1) << 20;
  static bool capturing(hipStream_t s) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (s == nullptr || hipStreamIsCapturing(s, &st) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return st == hipStreamCaptureStatusActive;
  }
  std::mutex mu_;
  std::multimap<size_t, Block> free_;
  std::map<void *, Block> live_;
  std::set<void *> graph_;  // captured (graph-owned) allocations
  size_t cached_ = 0;       // bytes in free_
  uint64_t tick_ = 0;
};

vs_status DeviceBuffer::alloc(size_t bytes, hipStream_t stream) {
  release();
  stream_ = stream;
  bytes_ = bytes;
  if (bytes == 0) return VS_OK;
  ptr_ = ScratchPool::get().alloc(bytes, stream);
  if (!ptr_) {
    bytes_ = 0;
    if (ScratchPool::refused_in_capture(bytes, stream)) {
      set_error("scratch of %zu bytes inside a stream capture is not supported (limit 1 MiB "
                "per allocation): run this call outside the captured region", bytes);
      return VS_ERR_UNSUPPORTED;
    }
    set_error("device allocation of %zu bytes failed", bytes);
    return VS_ERR_ALLOC;
  }
  return VS_OK;
}

void DeviceBuffer::release() {
  if (ptr_) ScratchPool::get().release(ptr_, stream_);
  ptr_ = nullptr;
  bytes_ = 0;
}

void release_cached_memory() { ScratchPool::get().release_all_free(); }
bool scratch_refused_in_capture(size_t bytes, hipStream_t stream) {
  return ScratchPool::refused_in_capture(bytes, stream);
}

// ------------------------------------------------------- packed staging
namespace {

// Per thread: a pinned, device-mapped host arena and a device arena of the
// same size.  Small operands of a call live in them for the duration of the
// call:
//   * zero-copy operands (read or written once per element, e.g. the
//     elementwise maps and every output): kernels access the pinned image
//     directly over the host link -- no DMA set-up at all;
//   * re-read inputs (convolution windows, GEMM panels, read by many
//     workgroups): packed into the pinned image and sent to the device
//     image with ONE host->device copy before the first kernel reads them.
// Staging every operand through its own pageable copy (HIP bounces
// each through an internal buffer) and ended with a blocking stream
// synchronise: ~40-65 us per call.
struct Arena {
  char *host = nullptr, *mapped = nullptr, *dev = nullptr;  // mapped = host, device view
  size_t cap = 0;
  int device = -1;
};

// Size of the image, per thread that calls the host API (VELES_STAGE_ARENA_MB).
size_t arena_bytes() {
  static const size_t v = static_cast<size_t>(env_int("VELES_STAGE_ARENA_MB", 16)) << 20;
  return v;
}
constexpr size_t kEagerFlush = 128 << 10;  // a packed input this large is sent at once

// Largest operand that is packed into the call's pinned image
// (VELES_STAGE_MAX_KB).
size_t stage_max() {
  static const size_t v = static_cast<size_t>(env_int("VELES_STAGE_MAX_KB", 4096)) << 10;
  return v;
}

constexpr size_t kPinnedInPlaceMin = 64 << 10;  // pinned operands above this skip the arena

// Images of threads that have ended wait here for the next thread that needs
// one: a program that calls the host API from short-lived threads holds as
// many images as it has such threads at once, not one per thread it ever
// started.  (No HIP call at thread exit: the main thread's exit may come
// after the HIP runtime has shut down.)  Never destroyed, so that a thread
// ending during process exit still finds it.
struct ArenaPool {
  std::mutex mu;
  std::vector<Arena> idle;
};
ArenaPool &arena_pool() {
  static ArenaPool *p = new ArenaPool;
  return *p;
}

struct ThreadArena : Arena {
  ~ThreadArena() {
    if (!host) return;
    ArenaPool &p = arena_pool();
    std::lock_guard<std::mutex> lock(p.mu);
    p.idle.push_back(*this);
  }
};

thread_local ThreadArena t_arena;
thread_local CallStaging *t_call = nullptr;

bool arena_ready() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  Arena &a = t_arena;
  if (a.host && a.device == dev) return true;
  if (arena_bytes() == 0) return false;  // VELES_STAGE_ARENA_MB=0: every operand by its own copy
  ArenaPool &pool = arena_pool();
  {
    std::lock_guard<std::mutex> lock(pool.mu);
    if (a.host) {  // this thread moved to another device
      pool.idle.push_back(a);
      a = Arena{};
    }
    for (size_t i = 0; i < pool.idle.size(); ++i)
      if (pool.idle[i].device == dev && pool.idle[i].cap == arena_bytes()) {
        a = pool.idle[i];
        pool.idle.erase(pool.idle.begin() + static_cast<long>(i));
        return true;
      }
  }
  void *h = nullptr, *m = nullptr, *d = nullptr;
  if (hipHostMalloc(&h, arena_bytes(), hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(&m, h, 0) != hipSuccess || hipMalloc(&d, arena_bytes()) != hipSuccess) {
    (void)hipGetLastError();
    if (h) (void)hipHostFree(h);
    return false;
  }
  a.host = static_cast<char *>(h);
  a.mapped = static_cast<char *>(m);
  a.dev = static_cast<char *>(d);
  a.cap = arena_bytes();
  a.device = dev;
  return true;
}

bool zero_copy_enabled() {
  static const bool v = env_int("VELES_ZERO_COPY", 1) != 0;
  return v;
}

}  // namespace

CallStaging::CallStaging(hipStream_t s) : stream_(s), prev_(t_call) { t_call = this; }
CallStaging::~CallStaging() { t_call = prev_; }
CallStaging *CallStaging::current() { return t_call; }

void *CallStaging::reserve(const void *host_in, size_t bytes, bool zero_copy) {
  if (bytes == 0 || bytes > stage_max()) return nullptr;
  const size_t off = (used_ + 255) & ~size_t{255};
  if (!arena_ready() || off + bytes > t_arena.cap) return nullptr;
  used_ = off + bytes;
  if (host_in) std::memcpy(t_arena.host + off, host_in, bytes);
  if (zero_copy && zero_copy_enabled()) return t_arena.mapped + off;
  if (host_in) {
    if (pend_hi_ == pend_lo_) pend_lo_ = off;
    pend_hi_ = off + bytes;
    // the DMA of a large operand runs while the host packs the next one
    if (bytes >= kEagerFlush) (void)flush();
  }
  return t_arena.dev + off;
}

vs_status CallStaging::flush() {
  if (pend_hi_ == pend_lo_) return VS_OK;
  const size_t lo = pend_lo_, n = pend_hi_ - pend_lo_;
  // a failed copy stays pending, so the flush before the first kernel reports it
  VS_HIP(hipMemcpyAsync(t_arena.dev + lo, t_arena.host + lo, n, hipMemcpyHostToDevice,
                        stream_));
  pend_lo_ = pend_hi_ = 0;
  return VS_OK;
}

void CallStaging::add_output(void *dev, void *host, size_t bytes) {
  char *p = static_cast<char *>(dev);
  const bool mapped = p >= t_arena.mapped && p < t_arena.mapped + t_arena.cap;
  outs_.push_back(Out{static_cast<size_t>(p - (mapped ? t_arena.mapped : t_arena.dev)), bytes,
                      host, mapped});
}

vs_status CallStaging::complete() {
  VS_TRY(flush());
  // device-image outputs (none unless zero-copy is off) come back first
  for (const Out &o : outs_)
    if (!o.mapped)
      VS_HIP(hipMemcpyAsync(t_arena.host + o.off, t_arena.dev + o.off, o.bytes,
                            hipMemcpyDeviceToHost, stream_));
  VS_TRY(wait_stream(stream_));
  for (const Out &o : outs_) std::memcpy(o.host, t_arena.host + o.off, o.bytes);
  outs_.clear();
  return VS_OK;
}

// Short waits (the common host-API case, ~10 us) are caught by polling: a
// blocking wait adds the wake-up latency of the interrupt path.  Past
// kSpinUs the wait is long enough not to care, and a blocking wait frees
// the core for other host threads.
vs_status wait_event(hipEvent_t ev) {
  constexpr long kSpinUs = 50;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e == hipSuccess) return VS_OK;
    if (e != hipErrorNotReady) return hip_status(e, "hipEventQuery", __FILE__, __LINE__);
    const auto us = std::chrono::duration_cast<std::chrono::microseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    if (us > kSpinUs) break;
  }
  VS_HIP(hipEventSynchronize(ev));
  return VS_OK;
}

namespace {
// Events of the calling thread on the current device: 0 for wait_stream, 1
// and 2 for the two halves of the staging image in pipelined_map.
vs_status thread_event(int which, hipEvent_t *out) {
  thread_local hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  thread_local int ev_dev = -1;
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (ev_dev != dev) {
    for (hipEvent_t &e : ev)
      if (e) {
        (void)hipEventDestroy(e);
        e = nullptr;
      }
    ev_dev = dev;
  }
  if (!ev[which]) VS_HIP(hipEventCreateWithFlags(&ev[which], hipEventDisableTiming));
  *out = ev[which];
  return VS_OK;
}
}  // namespace

vs_status wait_stream(hipStream_t s) {
  hipEvent_t ev = nullptr;
  VS_TRY(thread_event(0, &ev));
  VS_HIP(hipEventRecord(ev, s));
  return wait_event(ev);
}

// What the runtime knows about a pointer: device memory, host memory it has
// pinned (hipHostMalloc: vs_host_alloc, torch pinned tensors) with the address the GPU maps it at, or plain
// pageable host memory.
enum class MemKind { kDevice, kPinned, kPageable };
static MemKind classify(const void *p, void **mapped) {
  *mapped = nullptr;
  if (!p || !gpu_available() || in_brk_heap(p)) return MemKind::kPageable;
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return MemKind::kPageable;
  }
  if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged)
    return MemKind::kDevice;
  if (attr.type == hipMemoryTypeHost && attr.devicePointer) {
    *mapped = attr.devicePointer;
    return MemKind::kPinned;
  }
  return MemKind::kPageable;
}

Staged::Staged(const void *user, size_t bytes, Dir dir, hipStream_t stream)
    : user_(const_cast<void *>(user)), bytes_(bytes), dir_(dir),
      stream_(stream) {
  void *mapped = nullptr;
  const MemKind kind = classify(user, &mapped);
  if (kind == MemKind::kDevice) {
    dev_ = user_;
    log(2, "stage %p (%zu B): device pointer, used in place", user, bytes);
    return;
  }
  // Pinned operands past the arena's per-operand limit skip the host copies
  // of the pageable path (a 1 MiB memcpy costs more than its PCIe transfer):
  // read-once inputs are read in place through the mapping, re-read inputs
  // and outputs move by asynchronous DMA -- truly asynchronous from pinned
  // memory; from pageable memory hipMemcpyAsync stages and blocks.
  if (kind == MemKind::kPinned && bytes > kPinnedInPlaceMin && !sync_stage()) {
    pinned_ = true;
    // read-once inputs and outputs use the mapping in place (an output
    // written through it overlaps the kernel: 300 x 256 x 1000 takes 82 us
    // against 98 us with a device buffer and a DMA back)
    if (dir == kIn || dir == kOut) {
      dev_ = mapped;
      log(2, "stage %p (%zu B): pinned input, read in place", user, bytes);
      return;
    }
    status_ = buf_.alloc(bytes, stream);
    if (status_ != VS_OK) return;
    dev_ = buf_.get();
    log(2, "stage %p (%zu B): pinned, DMA dir=%d", user, bytes, static_cast<int>(dir));
    if (dir & kIn) {
      const hipError_t e = hipMemcpyAsync(dev_, user_, bytes, hipMemcpyHostToDevice, stream);
      if (e != hipSuccess)
        status_ = hip_status(e, "stage-in hipMemcpyAsync (pinned)", __FILE__, __LINE__);
    }
    return;
  }
  log(2, "stage %p (%zu B): host buffer, dir=%d", user, bytes, static_cast<int>(dir));
  if (CallStaging *cs = CallStaging::current(); cs && !sync_stage()) {
    // inputs re-read by many workgroups go to device memory; outputs and
    // read-once inputs stay in the mapped host image
    const bool zero_copy = !(dir & kIn) || !(dir & kReread);
    if (void *d = cs->reserve((dir & kIn) ? user : nullptr, bytes, zero_copy)) {
      dev_ = d;
      packed_ = true;
      return;
    }
  }
  status_ = buf_.alloc(bytes, stream);
  if (status_ != VS_OK) return;
  dev_ = buf_.get();
  if ((dir & kIn) && bytes) {
    hipError_t e =
        sync_stage()
            ? hipMemcpyWithStream(dev_, user_, bytes, hipMemcpyHostToDevice, stream)
            : hipMemcpyAsync(dev_, user_, bytes, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess)
      status_ = hip_status(e, "stage-in hipMemcpyAsync", __FILE__, __LINE__);
  }
}

vs_status Staged::finish() {
  if (status_ != VS_OK) return status_;
  if (dev_ == user_ || !(dir_ & kOut) || !bytes_) return VS_OK;
  if (pinned_) {  // asynchronous; the call's final wait covers it
    if (!buf_.get()) return VS_OK;  // written in place through the mapping
    VS_HIP(hipMemcpyAsync(user_, dev_, bytes_, hipMemcpyDeviceToHost, stream_));
    return VS_OK;
  }
  if (packed_) {
    CallStaging::current()->add_output(dev_, user_, bytes_);
    return VS_OK;
  }
  if (sync_stage())
    VS_HIP(hipMemcpyWithStream(user_, dev_, bytes_, hipMemcpyDeviceToHost, stream_));
  else
    VS_HIP(hipMemcpyAsync(user_, dev_, bytes_, hipMemcpyDeviceToHost, stream_));
  return VS_OK;
}

bool stage_image(StageImage *out) {
  static const bool enabled = env_int("VELES_PIPELINED_MAP", 1) != 0;
  if (!enabled || sync_stage() || !zero_copy_enabled() || !arena_ready()) return false;
  const Arena &a = t_arena;
  *out = StageImage{a.host, a.mapped, a.dev, a.cap};
  return true;
}

bool is_pageable_host(const void *p) {
  void *mapped = nullptr;
  return classify(p, &mapped) == MemKind::kPageable;
}

vs_status stage_half_event(int half, hipEvent_t *ev) { return thread_event(1 + (half & 1), ev); }

bool pipelined_map(hipStream_t s, size_t n, const MapArray *arrays, int count,
                   const MapLaunch &launch, vs_status *status) {
  // 1 MiB of floats per array and piece (0.25 to 2 MiB measure within noise of
  // each other)
  constexpr size_t kPieceElems = 256 << 10;
  constexpr int kMaxArrays = 8;
  *status = VS_OK;
  StageImage img;
  if (n < 2 * kPieceElems || count > kMaxArrays) return false;
  size_t per_elem = 0;
  for (int i = 0; i < count; i++) {
    void *mapped = nullptr;
    const void *p = arrays[i].in ? arrays[i].in : arrays[i].out;
    if (classify(p, &mapped) != MemKind::kPageable) return false;
    per_elem += arrays[i].elem;
  }
  if (per_elem == 0 || !stage_image(&img)) return false;
  const struct { char *host, *mapped; size_t cap; } a = {img.host, img.mapped, img.bytes};
  const size_t half = a.cap / 2;
  if (half <= 256 * static_cast<size_t>(count)) return false;
  size_t piece = kPieceElems;
  const size_t fit = (half - 256 * static_cast<size_t>(count)) / per_elem;
  if (fit < piece) piece = fit & ~size_t{63};
  if (piece == 0) return false;
  // offsets of the arrays inside one half
  size_t off[kMaxArrays];
  size_t cur = 0;
  for (int i = 0; i < count; i++) {
    off[i] = cur;
    cur += (piece * arrays[i].elem + 255) & ~size_t{255};
  }
  hipEvent_t ev[2] = {nullptr, nullptr};
  if ((*status = thread_event(1, &ev[0])) != VS_OK) return true;
  if ((*status = thread_event(2, &ev[1])) != VS_OK) return true;
  const size_t pieces = (n + piece - 1) / piece;
  log(2, "pipelined map: %zu elements in %zu pieces of %zu", n, pieces, piece);
  // step c: retire piece c - 2 (same half), then fill and launch piece c
  for (size_t c = 0; c < pieces + 2; c++) {
    const size_t h = (c & 1) * half;
    if (c >= 2) {
      const size_t first = (c - 2) * piece, cnt = std::min(piece, n - first);
      if ((*status = wait_event(ev[c & 1])) != VS_OK) break;
      for (int i = 0; i < count; i++)
        if (arrays[i].out)
          std::memcpy(static_cast<char *>(arrays[i].out) + first * arrays[i].elem,
                      a.host + h + off[i], cnt * arrays[i].elem);
    }
    if (c < pieces) {
      const size_t first = c * piece, cnt = std::min(piece, n - first);
      void *dev[kMaxArrays];
      for (int i = 0; i < count; i++) {
        if (arrays[i].in)
          std::memcpy(a.host + h + off[i],
                      static_cast<const char *>(arrays[i].in) + first * arrays[i].elem,
                      cnt * arrays[i].elem);
        dev[i] = a.mapped + h + off[i];
      }
      if ((*status = launch(dev, cnt, s)) != VS_OK) break;
      const hipError_t e = hipEventRecord(ev[c & 1], s);
      if (e != hipSuccess) {
        *status = hip_status(e, "hipEventRecord", __FILE__, __LINE__);
        break;
      }
    }
  }
  // on an error, nothing may still be using the image when the caller goes on
  if (*status != VS_OK) (void)hipStreamSynchronize(s);
  return true;
}

}  // namespace vs

extern "C" {

const char *vs_version(void) { return "0.1.0"; }
int vs_gpu_available(void) { return vs::gpu_available() ? 1 : 0; }
int vs_device_count(void) { return vs::device_count(); }
int vs_set_device(int device) {
  if (device < 0 || device >= vs::device_count()) {
    vs::set_error("vs_set_device(%d): %d device(s) visible", device,
                  vs::device_count());
    return VS_ERR_INVALID;
  }
  VS_HIP(hipSetDevice(device));
  return VS_OK;
}
int vs_get_device(void) {
  int d = -1;
  if (!vs::gpu_available() || hipGetDevice(&d) != hipSuccess) return -1;
  return d;
}
const char *vs_last_error(void) { return vs::last_error(); }
int vs_is_device_pointer(const void *ptr) {
  return vs::is_device_pointer(ptr) ? 1 : 0;
}
vs_status vs_stream_synchronize(vs_stream_t stream) {
  VS_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  return VS_OK;
}
int vs_compiled_arch(void) { return 950; }

void *vs_host_alloc(size_t bytes) {
  void *p = nullptr;
  if (!vs::gpu_available() || bytes == 0) return nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    vs::set_error("vs_host_alloc: %zu bytes of pinned memory failed", bytes);
    return nullptr;
  }
  return p;
}
void vs_host_free(void *p) {
  if (p) (void)hipHostFree(p);
}
void vs_release_cached_memory(void) { vs::release_cached_memory(); }

}  // extern "C"
