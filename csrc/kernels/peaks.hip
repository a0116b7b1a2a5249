// Strict-extremum detection with ordered compaction.
//
// x[i], 1 <= i <= n-2, is an extremum when (x[i]-x[i-1]) (x[i]-x[i+1]) > 0
// (reference src/detect_peaks.c:41-56).  Three passes, no atomics, results in
// increasing position order:
//   1. every 256-thread block counts the extrema of its 4096-sample chunk
//      (wavefront ballots + popcount);
//   2. one block turns the counts into exclusive offsets;
//   3. every block re-flags its chunk and writes positions/values at
//      offset + (rank inside the block), ranks from ballot prefix counts.
// The reference grows its result with realloc per element (:19-39); here the
// host API reads the total first and allocates the result once.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csrc/runtime/runtime.h"
#include "simd/detect_peaks.h"
#include "simd/gpu.h"

namespace vs {
namespace peaks {
namespace {

constexpr int kThreads = 256;
constexpr int kPer = 16;
constexpr int kChunk = kThreads * kPer;

__device__ __forceinline__ bool is_peak(const float *__restrict__ x, long long i,
                                        long long n, int type) {
  if (i < 1 || i >= n - 1) return false;
  const float c = x[i];
  const float d1 = c - x[i - 1];
  const float d2 = c - x[i + 1];
  if (!(d1 * d2 > 0.f)) return false;
  return (d1 > 0.f && (type & kExtremumTypeMaximum)) ||
         (d1 < 0.f && (type & kExtremumTypeMinimum));
}

// Sample i of round r handled by thread t: i = chunk0 + r * 256 + t, so a
// wavefront's 64 lanes test 64 consecutive samples (coalesced) per round.
__global__ __launch_bounds__(kThreads) void count_kernel(
    const float *__restrict__ x, long long n, int type,
    unsigned *__restrict__ counts) {
  __shared__ unsigned wsum[kThreads / 64];
  const long long c0 = static_cast<long long>(blockIdx.x) * kChunk;
  unsigned cnt = 0;
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    const bool p = is_peak(x, c0 + r * kThreads + threadIdx.x, n, type);
    cnt += __popcll(__ballot(p));
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) wsum[wid] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned s = 0;
    for (int w = 0; w < kThreads / 64; w++) s += wsum[w];
    counts[blockIdx.x] = s;
  }
}

// Exclusive scan of `nb` counts by one block; total to *total.
__global__ __launch_bounds__(1024) void scan_kernel(
    unsigned *__restrict__ counts, long long nb,
    unsigned long long *__restrict__ total) {
  __shared__ unsigned long long part[1024];
  // each thread scans a contiguous run
  const long long per = (nb + 1023) / 1024;
  const long long b0 = threadIdx.x * per;
  unsigned long long s = 0;
  for (long long b = b0; b < b0 + per && b < nb; b++) s += counts[b];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    unsigned long long v = threadIdx.x >= static_cast<unsigned>(off) ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  unsigned long long run = threadIdx.x ? part[threadIdx.x - 1] : 0;
  for (long long b = b0; b < b0 + per && b < nb; b++) {
    const unsigned c = counts[b];
    counts[b] = static_cast<unsigned>(run);  // offsets fit 32 bits: n < 2^32
    run += c;
  }
  if (threadIdx.x == 1023) *total = part[1023];
}

__global__ __launch_bounds__(kThreads) void emit_kernel(
    const float *__restrict__ x, long long n, int type,
    const unsigned *__restrict__ offsets, int *__restrict__ pos,
    float *__restrict__ val, unsigned long long cap) {
  __shared__ unsigned wbase[kPer][kThreads / 64];
  const long long c0 = static_cast<long long>(blockIdx.x) * kChunk;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  bool flag[kPer];
  unsigned long long masks[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    flag[r] = is_peak(x, c0 + r * kThreads + threadIdx.x, n, type);
    masks[r] = __ballot(flag[r]);
    if (lane == 0) wbase[r][wid] = __popcll(masks[r]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // order: round-major, then wavefront
    unsigned run = offsets[blockIdx.x];
    for (int r = 0; r < kPer; r++)
      for (int w = 0; w < kThreads / 64; w++) {
        const unsigned c = wbase[r][w];
        wbase[r][w] = run;
        run += c;
      }
  }
  __syncthreads();
  const unsigned long long below = (1ULL << lane) - 1ULL;
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    if (!flag[r]) continue;
    const unsigned long long slot = wbase[r][wid] + __popcll(masks[r] & below);
    if (slot < cap) {
      const long long i = c0 + r * kThreads + threadIdx.x;
      pos[slot] = static_cast<int>(i);
      val[slot] = x[i];
    }
  }
}

// Vector variant (x 16-byte aligned): each lane loads one float4 (4
// consecutive samples) per round, its neighbours' edge samples arrive by
// lane shuffles (lane 0 / 63 of a wave load the sample across the wave
// boundary), so every sample is loaded once instead of three times.  Round r
// of thread t covers samples c0 + 1024 r + 4 t + e, e < 4: positions stay in
// (round, wave, lane, e) order.  Flags of a lane are a 4-bit set; in-wave
// ranks come from ballots of the bits of each lane's flag count.
constexpr int kPer4 = kChunk / (4 * kThreads);  // rounds per block (same chunk)

__device__ __forceinline__ unsigned flags4(const float *__restrict__ x, long long i0,
                                           long long n, int type) {
  float4 v;
  if (i0 + 3 < n) {
    v = *reinterpret_cast<const float4 *>(x + i0);
  } else {
    v.x = i0 < n ? x[i0] : 0.f;
    v.y = i0 + 1 < n ? x[i0 + 1] : 0.f;
    v.z = i0 + 2 < n ? x[i0 + 2] : 0.f;
    v.w = i0 + 3 < n ? x[i0 + 3] : 0.f;
  }
  const int lane = threadIdx.x & 63;
  float prev = __shfl_up(v.w, 1);
  float next = __shfl_down(v.x, 1);
  if (lane == 0) prev = i0 >= 1 && i0 - 1 < n ? x[i0 - 1] : 0.f;
  if (lane == 63) next = i0 + 4 < n ? x[i0 + 4] : 0.f;
  const float s[6] = {prev, v.x, v.y, v.z, v.w, next};
  unsigned f = 0;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const long long i = i0 + e;
    const float c = s[e + 1];
    const float d1 = c - s[e];
    const float d2 = c - s[e + 2];
    const bool p = i >= 1 && i < n - 1 && d1 * d2 > 0.f &&
                   ((d1 > 0.f && (type & kExtremumTypeMaximum)) ||
                    (d1 < 0.f && (type & kExtremumTypeMinimum)));
    f |= p ? (1u << e) : 0u;
  }
  return f;
}

__global__ __launch_bounds__(kThreads) void count4_kernel(
    const float *__restrict__ x, long long n, int type, unsigned *__restrict__ counts) {
  __shared__ unsigned wsum[kThreads / 64];
  const long long c0 = static_cast<long long>(blockIdx.x) * kChunk;
  unsigned cnt = 0;
#pragma unroll
  for (int r = 0; r < kPer4; r++)
    cnt += __popc(flags4(x, c0 + r * 4 * kThreads + 4 * threadIdx.x, n, type));
  // wave sum of the per-lane counts
  for (int off = 32; off > 0; off >>= 1) cnt += __shfl_xor(cnt, off);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) wsum[wid] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned s = 0;
    for (int w = 0; w < kThreads / 64; w++) s += wsum[w];
    counts[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(kThreads) void emit4_kernel(
    const float *__restrict__ x, long long n, int type,
    const unsigned *__restrict__ offsets, int *__restrict__ pos,
    float *__restrict__ val, unsigned long long cap) {
  __shared__ unsigned wbase[kPer4][kThreads / 64], wcnt[kPer4][kThreads / 64];
  // per-wave staging of one round's results (<= 256 per wave), written out
  // as one contiguous run per wave (lanes' own slots are up to 4 apart: the
  // direct stores were scattered)
  __shared__ int spos[kThreads / 64][4 * 64];
  __shared__ float sval[kThreads / 64][4 * 64];
  const long long c0 = static_cast<long long>(blockIdx.x) * kChunk;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long below = (1ULL << lane) - 1ULL;
  unsigned f[kPer4], rank[kPer4];
#pragma unroll
  for (int r = 0; r < kPer4; r++) {
    f[r] = flags4(x, c0 + r * 4 * kThreads + 4 * threadIdx.x, n, type);
    const unsigned c = __popc(f[r]);  // 0..4: three bits
    const unsigned long long b0 = __ballot(c & 1u), b1 = __ballot(c & 2u),
                             b2 = __ballot(c & 4u);
    rank[r] = __popcll(b0 & below) + 2 * __popcll(b1 & below) + 4 * __popcll(b2 & below);
    if (lane == 0) wcnt[r][wid] = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // order: round-major, then wavefront
    unsigned run = offsets[blockIdx.x];
    for (int r = 0; r < kPer4; r++)
      for (int w = 0; w < kThreads / 64; w++) {
        wbase[r][w] = run;
        run += wcnt[r][w];
      }
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kPer4; r++) {
    const long long i0 = c0 + r * 4 * kThreads + 4 * threadIdx.x;
    unsigned k = rank[r];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      if (f[r] & (1u << e)) {
        spos[wid][k] = static_cast<int>(i0 + e);
        sval[wid][k] = x[i0 + e];
        k++;
      }
    }
    __syncthreads();
    const unsigned long long base = wbase[r][wid];
    const unsigned cnt = wcnt[r][wid];
    for (unsigned j = lane; j < cnt; j += 64) {
      if (base + j < cap) {
        pos[base + j] = spos[wid][j];
        val[base + j] = sval[wid][j];
      }
    }
    __syncthreads();
  }
}

}  // namespace
}  // namespace peaks
}  // namespace vs

using namespace vs;

extern "C" {

vs_status vs_detect_peaks(const float *x, size_t n, int type, int *pos,
                          float *val, size_t cap, unsigned long long *count,
                          vs_stream_t stream) {
  VS_REQUIRE(x && count, "vs_detect_peaks: null pointer");
  VS_REQUIRE(cap == 0 || (pos && val), "vs_detect_peaks: null output arrays");
  VS_REQUIRE(n >= 3 && n < (1ULL << 31), "vs_detect_peaks: size %zu out of range", n);
  VS_REQUIRE(type >= 1 && type <= 3, "vs_detect_peaks: bad extremum type %d", type);
  auto s = static_cast<hipStream_t>(stream);
  const long long nb = (static_cast<long long>(n) + peaks::kChunk - 1) / peaks::kChunk;
  DeviceBuffer counts;
  VS_TRY(counts.alloc(nb * sizeof(unsigned), s));
  // float4 path for 16-byte aligned x (each sample loaded once, not three
  // times: 2.1 TB/s before at 2^26, tools/bench_memops.py)
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(peaks::count4_kernel, dim3(static_cast<unsigned>(nb)),
                       dim3(peaks::kThreads), 0, s, x, static_cast<long long>(n), type,
                       counts.as<unsigned>());
  else
    hipLaunchKernelGGL(peaks::count_kernel, dim3(static_cast<unsigned>(nb)),
                       dim3(peaks::kThreads), 0, s, x, static_cast<long long>(n), type,
                       counts.as<unsigned>());
  hipLaunchKernelGGL(peaks::scan_kernel, dim3(1), dim3(1024), 0, s,
                     counts.as<unsigned>(), nb, count);
  if (cap > 0 && vec)
    hipLaunchKernelGGL(peaks::emit4_kernel, dim3(static_cast<unsigned>(nb)),
                       dim3(peaks::kThreads), 0, s, x, static_cast<long long>(n), type,
                       counts.as<unsigned>(), pos, val,
                       static_cast<unsigned long long>(cap));
  else if (cap > 0)
    hipLaunchKernelGGL(peaks::emit_kernel, dim3(static_cast<unsigned>(nb)),
                       dim3(peaks::kThreads), 0, s, x, static_cast<long long>(n), type,
                       counts.as<unsigned>(), pos, val,
                       static_cast<unsigned long long>(cap));
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // extern "C"
