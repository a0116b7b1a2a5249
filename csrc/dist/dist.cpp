// Multi-GPU layer of the C library (include/simd/dist.h).
//
// One process drives all ranks.  Each rank = (device, main stream, side
// stream).  Two backends implement the same collectives:
//   RCCL  -- ncclCommInitAll over distinct devices; collectives are enqueued
//            for all ranks inside one ncclGroupStart/End (single thread).
//            Over xGMI every pair of MI355X is one hop, so the halo exchange
//            is a set of concurrent neighbour send/recv pairs and the
//            all-gather runs on RCCL's own ring/direct algorithms.
//   LOCAL  -- stream-ordered peer / device-to-device copies with events;
//            several ranks may live on one device.  Used when RCCL cannot
//            form a communicator (shared devices, one GPU) and as the
//            test double that exercises every sharding / halo path on a
//            single GPU box (tests/test_dist.py).
// The reference has no distributed code at all (no such symbols); these entry points are new, shaped after its single-device
// APIs (src/convolve.c:381-395, src/wavelet.c:1907-1940, src/matrix.c:255).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/dist.h"

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "csrc/runtime/runtime.h"
#include "simd/wavelet_types.h"

struct vs_dist_context {
  int n = 0;
  int backend = VS_DIST_LOCAL;
  int timeout_ms = 300000;
  bool aborted = false;
  std::vector<int> dev;
  std::vector<hipStream_t> main, side;
  std::vector<ncclComm_t> comms;
};

namespace vs {
namespace dist {
namespace {

class DevGuard {
 public:
  explicit DevGuard(int d) {
    (void)hipGetDevice(&old_);
    (void)hipSetDevice(d);
  }
  ~DevGuard() { (void)hipSetDevice(old_); }

 private:
  int old_ = 0;
};

#define VS_NCCL(expr)                                                        \
  do {                                                                       \
    ncclResult_t vs_r_ = (expr);                                             \
    if (vs_r_ != ncclSuccess && vs_r_ != ncclInProgress) {                   \
      ::vs::set_error("%s: %s", #expr, ncclGetErrorString(vs_r_));           \
      return VS_ERR_COMM;                                                    \
    }                                                                        \
  } while (0)

// Per-rank events for LOCAL-backend ordering (created on the rank's device).
class Events {
 public:
  Events(vs_dist_context *c) : c_(c), ev_(c->n, nullptr) {}
  ~Events() {
    for (int r = 0; r < c_->n; r++)
      if (ev_[r]) (void)hipEventDestroy(ev_[r]);
  }
  vs_status record(const std::vector<hipStream_t> &s) {
    for (int r = 0; r < c_->n; r++) {
      DevGuard g(c_->dev[r]);
      if (!ev_[r]) VS_HIP(hipEventCreateWithFlags(&ev_[r], hipEventDisableTiming));
      VS_HIP(hipEventRecord(ev_[r], s[r]));
    }
    return VS_OK;
  }
  // stream s waits for rank q's recorded event
  vs_status wait(hipStream_t s, int q) {
    VS_HIP(hipStreamWaitEvent(s, ev_[q], 0));
    return VS_OK;
  }
  vs_status wait_all(hipStream_t s) {
    for (int q = 0; q < c_->n; q++) VS_TRY(wait(s, q));
    return VS_OK;
  }

 private:
  vs_dist_context *c_;
  std::vector<hipEvent_t> ev_;
};

vs_status copy(vs_dist_context *c, void *dst, int rd, const void *src, int rs,
               size_t bytes, hipStream_t s) {
  if (bytes == 0) return VS_OK;
  if (c->dev[rd] == c->dev[rs]) {
    VS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
  } else {
    VS_HIP(hipMemcpyPeerAsync(dst, c->dev[rd], src, c->dev[rs], bytes, s));
  }
  return VS_OK;
}

// A collective is complete on every stream of `s` once it returns (LOCAL:
// each stream waits for every rank's copies, matching RCCL's semantics that
// a rank's buffers are free again after its stream passes the collective).
vs_status local_fence(vs_dist_context *c, const std::vector<hipStream_t> &s) {
  Events done(c);
  VS_TRY(done.record(s));
  for (int r = 0; r < c->n; r++) {
    DevGuard g(c->dev[r]);
    VS_TRY(done.wait_all(s[r]));
  }
  return VS_OK;
}

vs_status broadcast_on(vs_dist_context *c, const std::vector<hipStream_t> &s,
                       void *const *bufs, size_t bytes, int root) {
  if (c->backend == VS_DIST_RCCL) {
    VS_NCCL(ncclGroupStart());
    for (int r = 0; r < c->n; r++) {
      DevGuard g(c->dev[r]);
      VS_NCCL(ncclBroadcast(bufs[r], bufs[r], bytes, ncclChar, root,
                            c->comms[r], s[r]));
    }
    VS_NCCL(ncclGroupEnd());
    return VS_OK;
  }
  Events ready(c);
  VS_TRY(ready.record(s));
  for (int r = 0; r < c->n; r++) {
    if (r == root) continue;
    DevGuard g(c->dev[r]);
    VS_TRY(ready.wait(s[r], root));
    VS_TRY(copy(c, bufs[r], r, bufs[root], root, bytes, s[r]));
  }
  return local_fence(c, s);
}

vs_status all_gather_on(vs_dist_context *c, const std::vector<hipStream_t> &s,
                        const void *const *send, void *const *recv, size_t bytes) {
  if (c->backend == VS_DIST_RCCL) {
    VS_NCCL(ncclGroupStart());
    for (int r = 0; r < c->n; r++) {
      DevGuard g(c->dev[r]);
      VS_NCCL(ncclAllGather(send[r], recv[r], bytes, ncclChar, c->comms[r], s[r]));
    }
    VS_NCCL(ncclGroupEnd());
    return VS_OK;
  }
  Events ready(c);
  VS_TRY(ready.record(s));
  for (int r = 0; r < c->n; r++) {
    DevGuard g(c->dev[r]);
    for (int q = 0; q < c->n; q++) {
      VS_TRY(ready.wait(s[r], q));
      VS_TRY(copy(c, static_cast<char *>(recv[r]) + q * bytes, r, send[q], q, bytes, s[r]));
    }
  }
  return local_fence(c, s);
}

// Variable-size all-gather in place: rank q's block of bytes[q] at offset
// off[q] of its buffer bufs[q] lands at the same offset of every rank's
// buffer.  RCCL: one group of in-place broadcasts, one per root (RCCL has
// no all-gatherv); over xGMI every root reaches every rank in one hop.
vs_status all_gatherv_on(vs_dist_context *c, const std::vector<hipStream_t> &s,
                         void *const *bufs, const size_t *off, const size_t *bytes) {
  if (c->backend == VS_DIST_RCCL) {
    VS_NCCL(ncclGroupStart());
    for (int q = 0; q < c->n; q++) {
      if (bytes[q] == 0) continue;
      for (int r = 0; r < c->n; r++) {
        DevGuard g(c->dev[r]);
        char *p = static_cast<char *>(bufs[r]) + off[q];
        VS_NCCL(ncclBroadcast(p, p, bytes[q], ncclChar, q, c->comms[r], s[r]));
      }
    }
    VS_NCCL(ncclGroupEnd());
    return VS_OK;
  }
  Events ready(c);
  VS_TRY(ready.record(s));
  for (int r = 0; r < c->n; r++) {
    DevGuard g(c->dev[r]);
    for (int q = 0; q < c->n; q++) {
      if (q == r || bytes[q] == 0) continue;
      VS_TRY(ready.wait(s[r], q));
      VS_TRY(copy(c, static_cast<char *>(bufs[r]) + off[q], r,
                  static_cast<const char *>(bufs[q]) + off[q], q, bytes[q], s[r]));
    }
  }
  return local_fence(c, s);
}

vs_status halo_on(vs_dist_context *c, const std::vector<hipStream_t> &s,
                  const float *const *src, const size_t *len, float *const *halo,
                  size_t h, int direction, int periodic) {
  const int n = c->n;
  if (h == 0) return VS_OK;
  for (int r = 0; r < n; r++)
    VS_REQUIRE(len[r] >= h, "vs_dist_halo_exchange: rank %d holds %zu < halo %zu samples",
               r, len[r], h);
  // peer[r]: the rank whose samples fill halo[r], -1 = zeros
  std::vector<int> peer(n);
  for (int r = 0; r < n; r++) {
    int q = direction > 0 ? r - 1 : r + 1;
    if (q < 0 || q >= n) q = periodic ? (q + n) % n : -1;
    peer[r] = q;
  }
  auto piece = [&](int q) {  // what rank q contributes
    return direction > 0 ? src[q] + (len[q] - h) : src[q];
  };
  const size_t bytes = h * sizeof(float);
  for (int r = 0; r < n; r++)
    if (peer[r] < 0) {
      DevGuard g(c->dev[r]);
      // a fill kernel, not a memset: callers may capture the stream
      VS_TRY(vs_fill(halo[r], 0.f, h, s[r]));
    }
  if (c->backend == VS_DIST_RCCL) {
    // self-exchange (periodic, one rank) is a local copy
    for (int r = 0; r < n; r++)
      if (peer[r] == r) {
        DevGuard g(c->dev[r]);
        VS_HIP(hipMemcpyAsync(halo[r], piece(r), bytes, hipMemcpyDeviceToDevice, s[r]));
      }
    VS_NCCL(ncclGroupStart());
    for (int r = 0; r < n; r++) {
      DevGuard g(c->dev[r]);
      if (peer[r] >= 0 && peer[r] != r)
        VS_NCCL(ncclRecv(halo[r], h, ncclFloat32, peer[r], c->comms[r], s[r]));
      for (int q = 0; q < n; q++)  // ranks that read from r
        if (q != r && peer[q] == r)
          VS_NCCL(ncclSend(piece(r), h, ncclFloat32, q, c->comms[r], s[r]));
    }
    VS_NCCL(ncclGroupEnd());
    return VS_OK;
  }
  Events ready(c);
  VS_TRY(ready.record(s));
  for (int r = 0; r < n; r++) {
    if (peer[r] < 0) continue;
    DevGuard g(c->dev[r]);
    VS_TRY(ready.wait(s[r], peer[r]));
    VS_TRY(copy(c, halo[r], r, piece(peer[r]), peer[r], bytes, s[r]));
  }
  return local_fence(c, s);
}

vs_status all_reduce_on(vs_dist_context *c, const std::vector<hipStream_t> &s,
                        float *const *bufs, size_t count) {
  if (c->backend == VS_DIST_RCCL) {
    VS_NCCL(ncclGroupStart());
    for (int r = 0; r < c->n; r++) {
      DevGuard g(c->dev[r]);
      VS_NCCL(ncclAllReduce(bufs[r], bufs[r], count, ncclFloat32, ncclSum, c->comms[r], s[r]));
    }
    VS_NCCL(ncclGroupEnd());
    return VS_OK;
  }
  // LOCAL: reduce into rank 0 through a scratch copy, then broadcast.
  if (c->n == 1) return VS_OK;
  Events ready(c);
  VS_TRY(ready.record(s));
  DevGuard g(c->dev[0]);
  DeviceBuffer tmp;
  VS_TRY(tmp.alloc(count * sizeof(float), s[0]));
  for (int q = 1; q < c->n; q++) {
    VS_TRY(ready.wait(s[0], q));
    VS_TRY(copy(c, tmp.get(), 0, bufs[q], q, count * sizeof(float), s[0]));
    VS_TRY(vs_binary(VS_OP_ADD, bufs[0], tmp.as<float>(), bufs[0], count, s[0]));
  }
  return broadcast_on(c, s, reinterpret_cast<void *const *>(bufs), count * sizeof(float), 0);
}

vs_status abort_all(vs_dist_context *c) {
  if (c->backend == VS_DIST_RCCL && !c->aborted)
    for (auto &cm : c->comms) (void)ncclCommAbort(cm);
  c->aborted = true;
  return VS_OK;
}

// Host pointer of upload/download (pageable or pinned, HIP stages).
vs_status h2d(int dev, void *dst, const void *src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return VS_OK;
  DevGuard g(dev);
  VS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s));
  return VS_OK;
}
vs_status d2h(int dev, void *dst, const void *src, size_t bytes, hipStream_t s) {
  if (bytes == 0) return VS_OK;
  DevGuard g(dev);
  VS_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
  return VS_OK;
}

// Per-rank scratch: buffers allocated on each rank's device / main stream.
struct RankBuffers {
  std::vector<DeviceBuffer> b;
  vs_status alloc(vs_dist_context *c, const std::vector<size_t> &bytes) {
    b.resize(c->n);
    for (int r = 0; r < c->n; r++) {
      DevGuard g(c->dev[r]);
      VS_TRY(b[r].alloc(std::max<size_t>(bytes[r], 4), c->main[r]));
    }
    return VS_OK;
  }
  vs_status alloc(vs_dist_context *c, size_t bytes) {
    return alloc(c, std::vector<size_t>(c->n, bytes));
  }
  float *f(int r) { return b[r].as<float>(); }
  std::vector<void *> ptrs() {
    std::vector<void *> p;
    for (auto &x : b) p.push_back(x.get());
    return p;
  }
};

// Events of one rank's call, destroyed with the list.
struct EventList {
  std::vector<hipEvent_t> ev;
  ~EventList() {
    for (auto e : ev)
      if (e) (void)hipEventDestroy(e);
  }
  vs_status record(hipStream_t s) {
    hipEvent_t e = nullptr;
    VS_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ev.push_back(e);
    VS_HIP(hipEventRecord(e, s));
    return VS_OK;
  }
};

// f(r) for every rank, each on a host thread of its own bound to the rank's
// device.  The sharded entry points take pageable host arrays, and a copy
// from or to pageable memory blocks the issuing thread until it is done: in
// one thread, rank r + 1's work would not even be enqueued before rank r's
// download has finished.  With one thread per rank every rank's copies and
// kernels are issued at once and the devices (and PCIe links) run side by
// side.  Collectives stay on the calling thread, between such phases.
template <class F>
vs_status for_ranks(vs_dist_context *c, F &&f) {
  if (c->n == 1) {
    DevGuard g(c->dev[0]);
    return f(0);
  }
  std::vector<vs_status> st(c->n, VS_OK);
  std::vector<std::string> err(c->n);
  std::vector<std::thread> th;
  th.reserve(c->n);
  for (int r = 0; r < c->n; r++)
    th.emplace_back([&, r] {
      DevGuard g(c->dev[r]);
      st[r] = f(r);
      if (st[r] != VS_OK) err[r] = last_error();
    });
  for (auto &t : th) t.join();
  for (int r = 0; r < c->n; r++)
    if (st[r] != VS_OK) {
      set_error("rank %d: %s", r, err[r].c_str());
      return st[r];
    }
  return VS_OK;
}

vs_status check_ctx(vs_dist_context *c) {
  VS_REQUIRE(c, "vs_dist: null context");
  VS_REQUIRE(!c->aborted, "vs_dist: communicator was aborted after an error");
  return VS_OK;
}

}  // namespace
}  // namespace dist
}  // namespace vs

using namespace vs;
using namespace vs::dist;

extern "C" {

void vs_dist_shard(size_t n, int nranks, int rank, size_t *begin, size_t *count) {
  if (nranks <= 0 || rank < 0 || rank >= nranks) {
    if (begin) *begin = 0;
    if (count) *count = 0;
    return;
  }
  const size_t q = n / nranks, rem = n % nranks;
  const size_t r = static_cast<size_t>(rank);
  if (begin) *begin = r * q + std::min(r, rem);
  if (count) *count = q + (r < rem ? 1 : 0);
}

vs_status vs_dist_create(int nranks, const int *devices, int backend, vs_dist_t *out) {
  clear_error();
  VS_REQUIRE(out, "vs_dist_create: null output");
  VS_REQUIRE(nranks >= 1 && nranks <= 1024, "vs_dist_create: bad rank count %d", nranks);
  VS_REQUIRE(backend >= VS_DIST_AUTO && backend <= VS_DIST_LOCAL,
             "vs_dist_create: bad backend %d", backend);
  if (!gpu_available()) {
    set_error("vs_dist_create: no usable gfx950 device");
    return VS_ERR_NO_GPU;
  }
  const int ndev = device_count();
  auto c = std::make_unique<vs_dist_context>();
  c->n = nranks;
  if (const char *e = std::getenv("VELES_DIST_TIMEOUT_MS")) c->timeout_ms = std::atoi(e);
  for (int r = 0; r < nranks; r++) {
    const int d = devices ? devices[r] : r % ndev;
    VS_REQUIRE(d >= 0 && d < ndev, "vs_dist_create: rank %d device %d of %d", r, d, ndev);
    c->dev.push_back(d);
  }
  std::vector<int> sorted = c->dev;
  std::sort(sorted.begin(), sorted.end());
  const bool distinct = std::adjacent_find(sorted.begin(), sorted.end()) == sorted.end();
  if (backend == VS_DIST_AUTO) backend = distinct ? VS_DIST_RCCL : VS_DIST_LOCAL;
  VS_REQUIRE(backend != VS_DIST_RCCL || distinct,
             "vs_dist_create: RCCL needs one rank per device");
  c->backend = backend;
  for (int r = 0; r < nranks; r++) {
    DevGuard g(c->dev[r]);
    hipStream_t a = nullptr, b = nullptr;
    VS_HIP(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
    VS_HIP(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
    c->main.push_back(a);
    c->side.push_back(b);
  }
  // Peer access lets LOCAL copies and kernels use xGMI directly.
  for (int r = 0; r < nranks; r++)
    for (int q = 0; q < nranks; q++)
      if (c->dev[r] != c->dev[q]) {
        DevGuard g(c->dev[r]);
        const hipError_t e = hipDeviceEnablePeerAccess(c->dev[q], 0);
        if (e != hipSuccess) (void)hipGetLastError();  // already enabled / none
      }
  if (backend == VS_DIST_RCCL) {
    c->comms.resize(nranks);
    const ncclResult_t st = ncclCommInitAll(c->comms.data(), nranks, c->dev.data());
    if (st != ncclSuccess) {
      set_error("ncclCommInitAll(%d): %s", nranks, ncclGetErrorString(st));
      for (int r = 0; r < nranks; r++) {
        (void)hipStreamDestroy(c->main[r]);
        (void)hipStreamDestroy(c->side[r]);
      }
      return VS_ERR_COMM;
    }
  }
  log(1, "vs_dist_create: %d ranks, backend %s", nranks,
      backend == VS_DIST_RCCL ? "rccl" : "local");
  *out = c.release();
  return VS_OK;
}

vs_status vs_dist_destroy(vs_dist_t c) {
  if (!c) return VS_OK;
  if (!c->aborted) (void)vs_dist_synchronize(c);
  for (auto &cm : c->comms)
    if (!c->aborted) (void)ncclCommDestroy(cm);
  for (int r = 0; r < c->n; r++) {
    DevGuard g(c->dev[r]);
    (void)hipStreamDestroy(c->main[r]);
    (void)hipStreamDestroy(c->side[r]);
  }
  delete c;
  return VS_OK;
}

int vs_dist_size(vs_dist_t c) { return c ? c->n : 0; }
int vs_dist_backend_of(vs_dist_t c) { return c ? c->backend : -1; }
int vs_dist_device(vs_dist_t c, int r) {
  return c && r >= 0 && r < c->n ? c->dev[r] : -1;
}
vs_stream_t vs_dist_stream(vs_dist_t c, int r) {
  return c && r >= 0 && r < c->n ? static_cast<vs_stream_t>(c->main[r]) : nullptr;
}

vs_status vs_dist_set_timeout(vs_dist_t c, int ms) {
  VS_TRY(check_ctx(c));
  VS_REQUIRE(ms >= 0, "vs_dist_set_timeout: negative timeout");
  c->timeout_ms = ms;
  return VS_OK;
}

vs_status vs_dist_synchronize(vs_dist_t c) {
  VS_TRY(check_ctx(c));
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    bool done = true;
    for (int r = 0; r < c->n; r++) {
      DevGuard g(c->dev[r]);
      for (hipStream_t s : {c->main[r], c->side[r]}) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipErrorNotReady) {
          done = false;
        } else if (e != hipSuccess) {
          abort_all(c);
          return hip_status(e, "hipStreamQuery (vs_dist_synchronize)", __FILE__, __LINE__);
        }
      }
      if (c->backend == VS_DIST_RCCL) {
        ncclResult_t st = ncclSuccess;
        (void)ncclCommGetAsyncError(c->comms[r], &st);
        if (st != ncclSuccess && st != ncclInProgress) {
          set_error("vs_dist: rank %d RCCL async error: %s", r, ncclGetErrorString(st));
          abort_all(c);
          return VS_ERR_COMM;
        }
      }
    }
    if (done) return VS_OK;
    const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    if (c->timeout_ms > 0 && ms > c->timeout_ms) {
      set_error("vs_dist_synchronize: timed out after %d ms", c->timeout_ms);
      abort_all(c);
      return VS_ERR_TIMEOUT;
    }
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

vs_status vs_dist_broadcast(vs_dist_t c, void *const *bufs, size_t bytes, int root) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(bufs && root >= 0 && root < c->n, "vs_dist_broadcast: bad arguments");
  return broadcast_on(c, c->main, bufs, bytes, root);
}

vs_status vs_dist_all_gather(vs_dist_t c, const void *const *send, void *const *recv,
                             size_t bytes) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(send && recv, "vs_dist_all_gather: null pointer");
  return all_gather_on(c, c->main, send, recv, bytes);
}

vs_status vs_dist_all_reduce_sum(vs_dist_t c, float *const *bufs, size_t n) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(bufs, "vs_dist_all_reduce_sum: null pointer");
  return all_reduce_on(c, c->main, bufs, n);
}

vs_status vs_dist_halo_exchange(vs_dist_t c, const float *const *src, const size_t *len,
                                float *const *halo, size_t h, int direction, int periodic) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(src && len && halo, "vs_dist_halo_exchange: null pointer");
  VS_REQUIRE(direction == 1 || direction == -1, "vs_dist_halo_exchange: direction must be +-1");
  return halo_on(c, c->main, src, len, halo, h, direction, periodic);
}

vs_status vs_dist_sgemm_rowsplit(vs_dist_t c, int m, int n, int k, const float *A,
                                 const float *B, float *C, int batch) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(A && B && C, "vs_dist_sgemm_rowsplit: null pointer");
  VS_REQUIRE(m > 0 && n > 0 && k > 0 && batch > 0, "vs_dist_sgemm_rowsplit: bad shape");
  const int R = c->n;
  std::vector<size_t> rb(R), rc(R);
  for (int r = 0; r < R; r++) vs_dist_shard(m, R, r, &rb[r], &rc[r]);
  const size_t kn = static_cast<size_t>(k) * n;
  // each rank holds only its rows of A and C and one copy of B
  RankBuffers dA, dB, dC;
  std::vector<size_t> abytes(R), cbytes(R);
  for (int r = 0; r < R; r++) {
    abytes[r] = batch * rc[r] * k * sizeof(float);
    cbytes[r] = batch * rc[r] * n * sizeof(float);
  }
  VS_TRY(dA.alloc(c, abytes));
  VS_TRY(dB.alloc(c, batch * kn * sizeof(float)));
  VS_TRY(dC.alloc(c, cbytes));
  // uploads: every rank's rows of A from its own host thread; B crosses
  // PCIe once (to rank 0) and reaches the other ranks over xGMI
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    for (int b = 0; b < batch; b++)
      VS_TRY(h2d(c->dev[r], dA.f(r) + b * rc[r] * k,
                 A + (static_cast<size_t>(b) * m + rb[r]) * k, rc[r] * k * sizeof(float),
                 c->main[r]));
    if (r == 0) VS_TRY(h2d(c->dev[0], dB.f(0), B, batch * kn * sizeof(float), c->main[0]));
    return VS_OK;
  }));
  {
    auto p = dB.ptrs();
    VS_TRY(broadcast_on(c, c->main, p.data(), batch * kn * sizeof(float), 0));
  }
  // per rank: every matrix's GEMM is enqueued on the main stream first (each
  // followed by an event), then the row blocks go straight to the caller's C
  // on the side stream, block b as soon as GEMM b has finished -- so the
  // download of matrix b overlaps GEMM b + 1, and the ranks' host threads
  // never wait for each other.  The host receives every row block from the
  // rank that computed it: no device needs the whole C, nothing is gathered.
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    if (rc[r] == 0) return VS_OK;
    EventList evs;
    for (int b = 0; b < batch; b++) {
      VS_TRY(vs_sgemm(0, 0, static_cast<int>(rc[r]), n, k, 1.f, dA.f(r) + b * rc[r] * k, k,
                      dB.f(r) + b * kn, n, 0.f, dC.f(r) + b * rc[r] * n, n, c->main[r]));
      VS_TRY(evs.record(c->main[r]));
    }
    for (int b = 0; b < batch; b++) {
      VS_HIP(hipStreamWaitEvent(c->side[r], evs.ev[b], 0));
      VS_TRY(d2h(c->dev[r], C + (static_cast<size_t>(b) * m + rb[r]) * n,
                 dC.f(r) + b * rc[r] * n, rc[r] * n * sizeof(float), c->side[r]));
    }
    VS_HIP(hipStreamSynchronize(c->side[r]));  // evs may go
    return VS_OK;
  }));
  return vs_dist_synchronize(c);
}

vs_status vs_dist_sgemm_rowsplit_device(vs_dist_t c, int m, int n, int k,
                                        const float *const *A, const float *const *B,
                                        float *const *C, int batch) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(A && B && C, "vs_dist_sgemm_rowsplit_device: null pointer");
  VS_REQUIRE(m > 0 && n > 0 && k > 0 && batch > 0, "vs_dist_sgemm_rowsplit_device: bad shape");
  const int R = c->n;
  std::vector<size_t> rb(R), rc(R);
  for (int r = 0; r < R; r++) vs_dist_shard(m, R, r, &rb[r], &rc[r]);
  for (int r = 0; r < R; r++)
    // a rank that owns no rows (m < ranks) has nothing to read from A
    VS_REQUIRE((A[r] || rc[r] == 0) && B[r] && C[r],
               "vs_dist_sgemm_rowsplit_device: rank %d null pointer", r);
  const size_t kn = static_cast<size_t>(k) * n, mn = static_cast<size_t>(m) * n;
  // matrix b: each rank writes its rows into its own full C, then the row
  // blocks are all-gathered in place on the side stream while the next
  // matrix's GEMM runs on the main stream
  std::vector<hipEvent_t> evs;
  struct EvFree {
    std::vector<hipEvent_t> *e;
    ~EvFree() {
      for (auto x : *e)
        if (x) (void)hipEventDestroy(x);
    }
  } evfree{&evs};
  std::vector<size_t> off(R), bytes(R);
  std::vector<void *> bufs(R);
  for (int b = 0; b < batch; b++) {
    for (int r = 0; r < R; r++) {
      DevGuard g(c->dev[r]);
      float *cb = C[r] + b * mn;
      if (rc[r] > 0)
        VS_TRY(vs_sgemm(0, 0, static_cast<int>(rc[r]), n, k, 1.f, A[r] + b * rc[r] * k, k,
                        B[r] + b * kn, n, 0.f, cb + rb[r] * n, n, c->main[r]));
      hipEvent_t ev = nullptr;
      VS_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      evs.push_back(ev);
      VS_HIP(hipEventRecord(ev, c->main[r]));
      VS_HIP(hipStreamWaitEvent(c->side[r], ev, 0));
      bufs[r] = cb;
      off[r] = rb[r] * n * sizeof(float);
      bytes[r] = rc[r] * n * sizeof(float);
    }
    VS_TRY(all_gatherv_on(c, c->side, bufs.data(), off.data(), bytes.data()));
  }
  // the caller's main streams see the gathered C
  Events gathered(c);
  VS_TRY(gathered.record(c->side));
  for (int r = 0; r < R; r++) {
    DevGuard g(c->dev[r]);
    VS_TRY(gathered.wait(c->main[r], r));
  }
  return VS_OK;
}

vs_status vs_dist_conv1d_batch(vs_dist_t c, int correlate, const float *x, int x_len,
                               const float *h, int h_len, float *y, int batch) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(x && h && y, "vs_dist_conv1d_batch: null pointer");
  VS_REQUIRE(x_len > 0 && h_len > 0 && batch > 0, "vs_dist_conv1d_batch: bad shape");
  const int R = c->n;
  const size_t ylen = static_cast<size_t>(x_len) + h_len - 1;
  std::vector<size_t> bb(R), bc(R);
  for (int r = 0; r < R; r++) vs_dist_shard(batch, R, r, &bb[r], &bc[r]);
  RankBuffers dx, dh, dy;
  std::vector<size_t> xb(R), yb(R);
  for (int r = 0; r < R; r++) {
    xb[r] = bc[r] * x_len * sizeof(float);
    yb[r] = bc[r] * ylen * sizeof(float);
  }
  VS_TRY(dx.alloc(c, xb));
  VS_TRY(dy.alloc(c, yb));
  VS_TRY(dh.alloc(c, h_len * sizeof(float)));
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    if (bc[r] == 0) return VS_OK;
    VS_TRY(h2d(c->dev[r], dx.f(r), x + bb[r] * x_len, xb[r], c->main[r]));
    VS_TRY(h2d(c->dev[r], dh.f(r), h, h_len * sizeof(float), c->main[r]));
    VS_TRY(vs_conv1d(VS_CONV_AUTO, correlate, dx.f(r), x_len, x_len, dh.f(r), h_len, 0,
                     dy.f(r), static_cast<int64_t>(ylen), static_cast<int>(bc[r]),
                     c->main[r]));
    return d2h(c->dev[r], y + bb[r] * ylen, dy.f(r), yb[r], c->main[r]);
  }));
  return vs_dist_synchronize(c);
}

// Data-parallel batches of the wavelet transforms and of independent GEMMs:
// rows (matrices) sharded over ranks with vs_dist_shard, no communication.
vs_status vs_dist_swt_batch(vs_dist_t c, int type, int order, int levels, int ext,
                            const float *x, int len, int batch, float *hi, float *lo) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(x && hi && lo, "vs_dist_swt_batch: null pointer");
  VS_REQUIRE(len > 0 && batch > 0 && levels >= 1, "vs_dist_swt_batch: bad shape");
  const int R = c->n;
  std::vector<size_t> bb(R), bc(R), xb(R), hb(R);
  for (int r = 0; r < R; r++) {
    vs_dist_shard(batch, R, r, &bb[r], &bc[r]);
    xb[r] = bc[r] * len * sizeof(float);
    hb[r] = xb[r] * levels;
  }
  RankBuffers dx, dhi, dlo;
  VS_TRY(dx.alloc(c, xb));
  VS_TRY(dhi.alloc(c, hb));
  VS_TRY(dlo.alloc(c, xb));
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    if (bc[r] == 0) return VS_OK;
    VS_TRY(h2d(c->dev[r], dx.f(r), x + bb[r] * len, xb[r], c->main[r]));
    VS_TRY(vs_swt_multilevel(type, order, levels, ext, dx.f(r), len, dhi.f(r), dlo.f(r),
                             static_cast<int>(bc[r]), c->main[r]));
    VS_TRY(d2h(c->dev[r], hi + bb[r] * levels * len, dhi.f(r), hb[r], c->main[r]));
    return d2h(c->dev[r], lo + bb[r] * len, dlo.f(r), xb[r], c->main[r]);
  }));
  return vs_dist_synchronize(c);
}

vs_status vs_dist_swt_batch_device(vs_dist_t c, int type, int order, int levels, int ext,
                                   const float *const *x, int len, const int *batch,
                                   float *const *hi, float *const *lo) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(x && hi && lo && batch, "vs_dist_swt_batch_device: null pointer");
  for (int r = 0; r < c->n; r++) {
    if (batch[r] == 0) continue;
    VS_REQUIRE(x[r] && hi[r] && lo[r], "vs_dist_swt_batch_device: rank %d null pointer", r);
    DevGuard g(c->dev[r]);
    VS_TRY(vs_swt_multilevel(type, order, levels, ext, x[r], len, hi[r], lo[r], batch[r],
                             c->main[r]));
  }
  return VS_OK;
}

vs_status vs_dist_dwt_batch(vs_dist_t c, int type, int order, int levels, int ext,
                            const float *x, int len, int batch, float *out) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(x && out, "vs_dist_dwt_batch: null pointer");
  VS_REQUIRE(len > 0 && batch > 0 && levels >= 1, "vs_dist_dwt_batch: bad shape");
  const int R = c->n;
  std::vector<size_t> bb(R), bc(R), xb(R);
  for (int r = 0; r < R; r++) {
    vs_dist_shard(batch, R, r, &bb[r], &bc[r]);
    xb[r] = bc[r] * len * sizeof(float);
  }
  RankBuffers dx, dout;
  VS_TRY(dx.alloc(c, xb));
  VS_TRY(dout.alloc(c, xb));
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    if (bc[r] == 0) return VS_OK;
    VS_TRY(h2d(c->dev[r], dx.f(r), x + bb[r] * len, xb[r], c->main[r]));
    VS_TRY(vs_dwt_multilevel(type, order, levels, ext, dx.f(r), len, dout.f(r),
                             static_cast<int>(bc[r]), c->main[r]));
    return d2h(c->dev[r], out + bb[r] * len, dout.f(r), xb[r], c->main[r]);
  }));
  return vs_dist_synchronize(c);
}

vs_status vs_dist_sgemm_batch(vs_dist_t c, int trans_a, int trans_b, int m, int n, int k,
                              const float *A, const float *B, float *C, int batch) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(A && B && C, "vs_dist_sgemm_batch: null pointer");
  VS_REQUIRE(m > 0 && n > 0 && k > 0 && batch > 0, "vs_dist_sgemm_batch: bad shape");
  const int R = c->n;
  const size_t mk = static_cast<size_t>(m) * k, kn = static_cast<size_t>(k) * n,
               mn = static_cast<size_t>(m) * n;
  std::vector<size_t> bb(R), bc(R), ab(R), bbytes(R), cb(R);
  for (int r = 0; r < R; r++) {
    vs_dist_shard(batch, R, r, &bb[r], &bc[r]);
    ab[r] = bc[r] * mk * sizeof(float);
    bbytes[r] = bc[r] * kn * sizeof(float);
    cb[r] = bc[r] * mn * sizeof(float);
  }
  RankBuffers dA, dB, dC;
  VS_TRY(dA.alloc(c, ab));
  VS_TRY(dB.alloc(c, bbytes));
  VS_TRY(dC.alloc(c, cb));
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    if (bc[r] == 0) return VS_OK;
    VS_TRY(h2d(c->dev[r], dA.f(r), A + bb[r] * mk, ab[r], c->main[r]));
    VS_TRY(h2d(c->dev[r], dB.f(r), B + bb[r] * kn, bbytes[r], c->main[r]));
    VS_TRY(vs_sgemm_strided_batched(trans_a, trans_b, m, n, k, 1.f, dA.f(r),
                                    trans_a ? m : k, static_cast<int64_t>(mk), dB.f(r),
                                    trans_b ? k : n, static_cast<int64_t>(kn), 0.f, dC.f(r), n,
                                    static_cast<int64_t>(mn), static_cast<int>(bc[r]),
                                    c->main[r]));
    return d2h(c->dev[r], C + bb[r] * mn, dC.f(r), cb[r], c->main[r]);
  }));
  return vs_dist_synchronize(c);
}

vs_status vs_dist_conv1d_long(vs_dist_t c, int correlate, const float *x, size_t x_len,
                              const float *h, int h_len, float *y) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(x && h && y, "vs_dist_conv1d_long: null pointer");
  VS_REQUIRE(x_len > 0 && h_len > 0, "vs_dist_conv1d_long: bad shape");
  const int R = c->n;
  const size_t H = h_len - 1;
  std::vector<size_t> b(R), cnt(R);
  for (int r = 0; r < R; r++) vs_dist_shard(x_len, R, r, &b[r], &cnt[r]);
  VS_REQUIRE(cnt[R - 1] >= H && cnt[R - 1] > 0,
             "vs_dist_conv1d_long: chunk %zu shorter than the filter history %zu "
             "(use fewer ranks)", cnt[R - 1], H);
  VS_REQUIRE(cnt[0] + H < (1ULL << 31), "vs_dist_conv1d_long: chunk too long");
  // xb[r] = [history H | chunk], yb[r] = full conv of xb[r]
  RankBuffers xb, yb, dh;
  std::vector<size_t> xs(R), ys(R);
  for (int r = 0; r < R; r++) {
    xs[r] = (H + cnt[r]) * sizeof(float);
    ys[r] = (H + cnt[r] + H) * sizeof(float);
  }
  VS_TRY(xb.alloc(c, xs));
  VS_TRY(yb.alloc(c, ys));
  VS_TRY(dh.alloc(c, h_len * sizeof(float)));
  std::vector<const float *> src(R);
  std::vector<float *> halo(R);
  for (int r = 0; r < R; r++) {
    src[r] = xb.f(r) + H;
    halo[r] = xb.f(r);
  }
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    VS_TRY(h2d(c->dev[r], xb.f(r) + H, x + b[r], cnt[r] * sizeof(float), c->main[r]));
    return h2d(c->dev[r], dh.f(r), h, h_len * sizeof(float), c->main[r]);
  }));
  VS_TRY(halo_on(c, c->main, src.data(), cnt.data(), halo.data(), H, +1, 0));
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    const int xl = static_cast<int>(H + cnt[r]);
    VS_TRY(vs_conv1d(VS_CONV_AUTO, correlate, xb.f(r), xl, xl, dh.f(r), h_len, 0, yb.f(r),
                     xl + h_len - 1, 1, c->main[r]));
    const size_t keep = cnt[r] + (r == R - 1 ? H : 0);
    return d2h(c->dev[r], y + b[r], yb.f(r) + H, keep * sizeof(float), c->main[r]);
  }));
  return vs_dist_synchronize(c);
}

vs_status vs_dist_swt_long(vs_dist_t c, int type, int order, int levels, int ext,
                           const float *x, size_t len, float *hi, float *lo) {
  clear_error();
  VS_TRY(check_ctx(c));
  VS_REQUIRE(x && hi && lo, "vs_dist_swt_long: null pointer");
  VS_REQUIRE(levels >= 1 && levels <= 24 && order >= 2, "vs_dist_swt_long: bad levels/order");
  const int R = c->n;
  const size_t Hmax = static_cast<size_t>(order - 1) << (levels - 1);
  std::vector<size_t> b(R), cnt(R);
  for (int r = 0; r < R; r++) vs_dist_shard(len, R, r, &b[r], &cnt[r]);
  VS_REQUIRE(cnt[R - 1] >= Hmax,
             "vs_dist_swt_long: chunk %zu shorter than the level-%d halo %zu (use fewer ranks)",
             cnt[R - 1], levels, Hmax);
  VS_REQUIRE(cnt[0] + Hmax < (1ULL << 31), "vs_dist_swt_long: chunk too long");
  const bool periodic = ext == EXTENSION_TYPE_PERIODIC;
  // cur[r] = [chunk | right halo], out hi/lo of the same length
  RankBuffers cur, ohi, olo;
  std::vector<size_t> sz(R);
  for (int r = 0; r < R; r++) sz[r] = (cnt[r] + Hmax) * sizeof(float);
  VS_TRY(cur.alloc(c, sz));
  {
    std::vector<size_t> two(R);
    for (int r = 0; r < R; r++) two[r] = 2 * sz[r];
    VS_TRY(ohi.alloc(c, two));
  }
  VS_TRY(olo.alloc(c, sz));
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    return h2d(c->dev[r], cur.f(r), x + b[r], cnt[r] * sizeof(float), c->main[r]);
  }));
  for (int l = 1; l <= levels; l++) {
    const size_t H = static_cast<size_t>(order - 1) << (l - 1);
    std::vector<const float *> src(R);
    std::vector<float *> halo(R);
    for (int r = 0; r < R; r++) {
      src[r] = cur.f(r);
      halo[r] = cur.f(r) + cnt[r];
    }
    // the last rank's halo only matters when periodic (else local extension)
    VS_TRY(halo_on(c, c->main, src.data(), cnt.data(), halo.data(), H, -1, periodic ? 1 : 0));
    // the level's kernel and the hand-over to the next level go on the main
    // stream; the band's download follows on the side stream, so it overlaps
    // the next level's halo exchange and kernel
    VS_TRY(for_ranks(c, [&](int r) -> vs_status {
      const bool local_ext = r == R - 1 && !periodic;
      const int n = static_cast<int>(local_ext ? cnt[r] : cnt[r] + H);
      // ohi alternates between two halves per level: level l's download may
      // still read its half while level l + 1's kernel writes the other
      float *oh = ohi.f(r) + (l & 1) * (cnt[r] + Hmax);
      VS_TRY(vs_swt(type, order, l, local_ext ? ext : EXTENSION_TYPE_ZERO, cur.f(r), n, n, oh,
                    olo.f(r), n, 1, c->main[r]));
      VS_HIP(hipMemcpyAsync(cur.f(r), olo.f(r), cnt[r] * sizeof(float),
                            hipMemcpyDeviceToDevice, c->main[r]));
      EventList done;
      VS_TRY(done.record(c->main[r]));
      VS_HIP(hipStreamWaitEvent(c->side[r], done.ev[0], 0));
      VS_TRY(d2h(c->dev[r], hi + (l - 1) * len + b[r], oh, cnt[r] * sizeof(float),
                 c->side[r]));
      VS_HIP(hipStreamSynchronize(c->side[r]));
      return VS_OK;
    }));
  }
  VS_TRY(for_ranks(c, [&](int r) -> vs_status {
    return d2h(c->dev[r], lo + b[r], cur.f(r), cnt[r] * sizeof(float), c->main[r]);
  }));
  return vs_dist_synchronize(c);
}

}  // extern "C"
