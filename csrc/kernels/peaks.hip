// Strict-extremum detection with ordered compaction, for one signal or a
// batch of rows in one launch sequence.
//
// x[i], 1 <= i <= n-2, is an extremum when (x[i]-x[i-1]) (x[i]-x[i+1]) > 0
// (reference src/detect_peaks.c:41-56).  Three passes, no atomics, results in
// increasing (row, position) order:
//   1. every 256-thread block counts the extrema of its 4096-sample chunk of
//      one row (wavefront ballots + popcount);
//   2. one block turns the counts into exclusive 64-bit offsets, and records
//      where every row's results start (a CSR row_start array);
//   3. every block re-flags its chunk and writes positions/values at
//      offset + (rank inside the block), ranks from ballot prefix counts.
// Positions are sample indices inside the row: int32, or int64 for rows of
// 2^31 samples and more (the reference's ExtremumPoint holds an int,
// inc/simd/detect_peaks.h:57-62, while its size argument is a size_t).
// The reference grows its result with realloc per element (:19-39); here the
// caller reads the totals first and allocates the result once.
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

// Block b works on chunk b % chunks_per_row of row b / chunks_per_row.
struct Rows {
  const float *x;
  long long n;       // samples per row
  long long stride;  // floats between rows
  long long cpr;     // chunks per row
  int type;
};

__device__ __forceinline__ void locate(const Rows &a, const float *&row, long long &c0) {
  const long long b = blockIdx.x, r = b / a.cpr;
  row = a.x + r * a.stride;
  c0 = (b - r * a.cpr) * kChunk;
}

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
__global__ __launch_bounds__(kThreads) void count_kernel(Rows a, unsigned *__restrict__ counts) {
  __shared__ unsigned wsum[kThreads / 64];
  const float *x;
  long long c0;
  locate(a, x, c0);
  unsigned cnt = 0;
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    const bool p = is_peak(x, c0 + r * kThreads + threadIdx.x, a.n, a.type);
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

// Exclusive scan of `nb` block counts by one block: offsets[b] (64-bit), and
// row_start[r] = offsets[r * cpr] for r < rows, row_start[rows] = total.
__global__ __launch_bounds__(1024) void scan_kernel(const unsigned *__restrict__ counts,
                                                    long long nb, long long cpr, long long rows,
                                                    unsigned long long *__restrict__ offsets,
                                                    unsigned long long *__restrict__ row_start) {
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
    offsets[b] = run;
    if (b % cpr == 0) row_start[b / cpr] = run;
    run += counts[b];
  }
  if (threadIdx.x == 1023) row_start[rows] = part[1023];
}

template <class POS>
__global__ __launch_bounds__(kThreads) void emit_kernel(
    Rows a, const unsigned long long *__restrict__ offsets, POS *__restrict__ pos,
    float *__restrict__ val, unsigned long long cap) {
  __shared__ unsigned wbase[kPer][kThreads / 64];
  const float *x;
  long long c0;
  locate(a, x, c0);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  bool flag[kPer];
  unsigned long long masks[kPer];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    flag[r] = is_peak(x, c0 + r * kThreads + threadIdx.x, a.n, a.type);
    masks[r] = __ballot(flag[r]);
    if (lane == 0) wbase[r][wid] = __popcll(masks[r]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // order: round-major, then wavefront
    unsigned run = 0;
    for (int r = 0; r < kPer; r++)
      for (int w = 0; w < kThreads / 64; w++) {
        const unsigned c = wbase[r][w];
        wbase[r][w] = run;
        run += c;
      }
  }
  __syncthreads();
  const unsigned long long below = (1ULL << lane) - 1ULL;
  const unsigned long long base = offsets[blockIdx.x];
#pragma unroll
  for (int r = 0; r < kPer; r++) {
    if (!flag[r]) continue;
    const unsigned long long slot = base + wbase[r][wid] + __popcll(masks[r] & below);
    if (slot < cap) {
      const long long i = c0 + r * kThreads + threadIdx.x;
      pos[slot] = static_cast<POS>(i);
      val[slot] = x[i];
    }
  }
}

// Vector variant (rows 16-byte aligned): each lane loads one float4 (4
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

__global__ __launch_bounds__(kThreads) void count4_kernel(Rows a, unsigned *__restrict__ counts) {
  __shared__ unsigned wsum[kThreads / 64];
  const float *x;
  long long c0;
  locate(a, x, c0);
  unsigned cnt = 0;
#pragma unroll
  for (int r = 0; r < kPer4; r++)
    cnt += __popc(flags4(x, c0 + r * 4 * kThreads + 4 * threadIdx.x, a.n, a.type));
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

template <class POS>
__global__ __launch_bounds__(kThreads) void emit4_kernel(
    Rows a, const unsigned long long *__restrict__ offsets, POS *__restrict__ pos,
    float *__restrict__ val, unsigned long long cap) {
  __shared__ unsigned wbase[kPer4][kThreads / 64], wcnt[kPer4][kThreads / 64];
  // per-wave staging of one round's results (<= 256 per wave), written out
  // as one contiguous run per wave (lanes' own slots are up to 4 apart: the
  // direct stores were scattered)
  __shared__ POS spos[kThreads / 64][4 * 64];
  __shared__ float sval[kThreads / 64][4 * 64];
  const float *x;
  long long c0;
  locate(a, x, c0);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const unsigned long long below = (1ULL << lane) - 1ULL;
  unsigned f[kPer4], rank[kPer4];
#pragma unroll
  for (int r = 0; r < kPer4; r++) {
    f[r] = flags4(x, c0 + r * 4 * kThreads + 4 * threadIdx.x, a.n, a.type);
    const unsigned c = __popc(f[r]);  // 0..4: three bits
    const unsigned long long b0 = __ballot(c & 1u), b1 = __ballot(c & 2u),
                             b2 = __ballot(c & 4u);
    rank[r] = __popcll(b0 & below) + 2 * __popcll(b1 & below) + 4 * __popcll(b2 & below);
    if (lane == 0) wcnt[r][wid] = __popcll(b0) + 2 * __popcll(b1) + 4 * __popcll(b2);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // order: round-major, then wavefront
    unsigned run = 0;
    for (int r = 0; r < kPer4; r++)
      for (int w = 0; w < kThreads / 64; w++) {
        wbase[r][w] = run;
        run += wcnt[r][w];
      }
  }
  __syncthreads();
  const unsigned long long block_base = offsets[blockIdx.x];
#pragma unroll
  for (int r = 0; r < kPer4; r++) {
    const long long i0 = c0 + r * 4 * kThreads + 4 * threadIdx.x;
    unsigned k = rank[r];
#pragma unroll
    for (int e = 0; e < 4; e++) {
      if (f[r] & (1u << e)) {
        spos[wid][k] = static_cast<POS>(i0 + e);
        sval[wid][k] = x[i0 + e];
        k++;
      }
    }
    __syncthreads();
    const unsigned long long base = block_base + wbase[r][wid];
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

// rows x n samples (row stride xs): counts -> offsets / row_start -> emit.
vs_status run(const float *x, size_t n, int64_t xs, size_t rows, int type, void *pos, int pos64,
              float *val, size_t cap, unsigned long long *row_start, hipStream_t s) {
  VS_REQUIRE(x && row_start, "vs_detect_peaks: null pointer");
  VS_REQUIRE(cap == 0 || (pos && val), "vs_detect_peaks: null output arrays");
  VS_REQUIRE(n >= 3, "vs_detect_peaks: size %zu out of range", n);
  VS_REQUIRE(pos64 || n < (1ULL << 31),
             "vs_detect_peaks: rows of %zu samples need 64-bit positions", n);
  VS_REQUIRE(type >= 1 && type <= 3, "vs_detect_peaks: bad extremum type %d", type);
  VS_REQUIRE(rows >= 1 && (rows == 1 || xs >= static_cast<int64_t>(n)),
             "vs_detect_peaks: bad row count / stride");
  const long long cpr = (static_cast<long long>(n) + kChunk - 1) / kChunk;
  const long long nb = cpr * static_cast<long long>(rows);
  VS_REQUIRE(nb < (1LL << 31), "vs_detect_peaks: %lld chunks exceed one launch", nb);
  DeviceBuffer counts, offsets;
  VS_TRY(counts.alloc(nb * sizeof(unsigned), s));
  VS_TRY(offsets.alloc(nb * sizeof(unsigned long long), s));
  const Rows a{x, static_cast<long long>(n), rows == 1 ? 0 : xs, cpr, type};
  // float4 path for 16-byte aligned rows (each sample loaded once, not three
  // times: 2.1 TB/s before at 2^26, tools/bench_memops.py)
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (rows == 1 || xs % 4 == 0);
  const dim3 grid(static_cast<unsigned>(nb)), block(kThreads);
  if (vec) hipLaunchKernelGGL(count4_kernel, grid, block, 0, s, a, counts.as<unsigned>());
  else hipLaunchKernelGGL(count_kernel, grid, block, 0, s, a, counts.as<unsigned>());
  hipLaunchKernelGGL(scan_kernel, dim3(1), dim3(1024), 0, s, counts.as<unsigned>(), nb, cpr,
                     static_cast<long long>(rows), offsets.as<unsigned long long>(), row_start);
  if (cap > 0) {
    const auto *off = offsets.as<unsigned long long>();
    const unsigned long long c = cap;
    if (vec && pos64)
      hipLaunchKernelGGL(emit4_kernel<long long>, grid, block, 0, s, a, off,
                         static_cast<long long *>(pos), val, c);
    else if (vec)
      hipLaunchKernelGGL(emit4_kernel<int>, grid, block, 0, s, a, off, static_cast<int *>(pos),
                         val, c);
    else if (pos64)
      hipLaunchKernelGGL(emit_kernel<long long>, grid, block, 0, s, a, off,
                         static_cast<long long *>(pos), val, c);
    else
      hipLaunchKernelGGL(emit_kernel<int>, grid, block, 0, s, a, off, static_cast<int *>(pos),
                         val, c);
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // namespace
}  // namespace peaks
}  // namespace vs

using namespace vs;

extern "C" {

vs_status vs_detect_peaks(const float *x, size_t n, int type, int *pos,
                          float *val, size_t cap, unsigned long long *count,
                          vs_stream_t stream) {
  VS_REQUIRE(count, "vs_detect_peaks: null pointer");
  auto s = static_cast<hipStream_t>(stream);
  // row_start of the one row: {0, total}; the caller's word receives the total
  DeviceBuffer rs;
  VS_TRY(rs.alloc(2 * sizeof(unsigned long long), s));
  VS_TRY(peaks::run(x, n, 0, 1, type, pos, 0, val, cap, rs.as<unsigned long long>(), s));
  VS_HIP(hipMemcpyAsync(count, rs.as<unsigned long long>() + 1, sizeof(unsigned long long),
                        hipMemcpyDefault, s));
  return VS_OK;
}

vs_status vs_detect_peaks_batched(const float *x, size_t n, int64_t x_stride, size_t rows,
                                  int type, void *pos, int pos64, float *val, size_t cap,
                                  unsigned long long *row_start, vs_stream_t stream) {
  return peaks::run(x, n, x_stride, rows, type, pos, pos64, val, cap, row_start,
                    static_cast<hipStream_t>(stream));
}

}  // extern "C"
