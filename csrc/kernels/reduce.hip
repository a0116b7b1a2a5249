// Reductions and uint8 normalisation.
//
// Deterministic two-pass reductions: pass 1 is a grid of at most 1024
// blocks, each reducing its grid-stride share with 16-byte loads, a
// wavefront butterfly (__shfl_xor over 64 lanes) and one LDS exchange; pass 2
// is a single block over the partials.  No float atomics: the result does
// not depend on dispatch order (cdna_hip_programming.md Guideline 12).
//
// Reference counterparts: inc/simd/arithmetic.h:791-808 (sum_elements),
// src/normalize.c:209-380 (SSE minmax / normalize bodies), :382-443 (scalar).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <algorithm>

#include <cfloat>
#include <cstdint>

#include "csrc/kernels/device.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace {

constexpr unsigned kBlock = 256;
constexpr unsigned kMaxPartials = 1024;

struct SumR {
  using T = float;
  __device__ static float init() { return 0.f; }
  __device__ static float op(float a, float b) { return a + b; }
  __device__ static float wave(float v) { return dev::wave_sum(v); }
};

// Block reduction of one value per thread; result valid in thread 0.
template <class R>
__device__ float block_reduce(float v) {
  __shared__ float part[kBlock / dev::kWave];
  v = R::wave(v);
  const int lane = threadIdx.x & (dev::kWave - 1), wid = threadIdx.x / dev::kWave;
  if (lane == 0) part[wid] = v;
  __syncthreads();
  v = R::init();
  if (threadIdx.x < blockDim.x / dev::kWave) v = part[threadIdx.x];
  if (wid == 0) v = R::wave(v);
  return v;
}

__global__ __launch_bounds__(kBlock) void sum_pass1(const float *__restrict__ x,
                                                    size_t n,
                                                    float *__restrict__ partial) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  float acc = 0.f;
  size_t done = 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const size_t n4 = n / 4;
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    for (size_t i = tid; i < n4; i += stride) {
      const float4 v = x4[i];
      acc += (v.x + v.y) + (v.z + v.w);
    }
    done = n4 * 4;
  }
  for (size_t i = done + tid; i < n; i += stride) acc += x[i];
  acc = block_reduce<SumR>(acc);
  if (threadIdx.x == 0) partial[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kBlock) void sum_pass2(const float *__restrict__ partial,
                                                    int np, float *__restrict__ out) {
  float acc = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) acc += partial[i];
  acc = block_reduce<SumR>(acc);
  if (threadIdx.x == 0) *out = acc;
}

__global__ __launch_bounds__(kBlock) void minmax_pass1(const float *__restrict__ x,
                                                       size_t n,
                                                       float2 *__restrict__ partial) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  float lo = FLT_MAX, hi = -FLT_MAX;
  // Seed with x[0] so an all-NaN-free array reproduces the scalar result.
  if (n) lo = hi = x[0];
  size_t done = 0;
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
    const size_t n4 = n / 4;
    const float4 *x4 = reinterpret_cast<const float4 *>(x);
    for (size_t i = tid; i < n4; i += stride) {
      const float4 v = x4[i];
      lo = fminf(lo, fminf(fminf(v.x, v.y), fminf(v.z, v.w)));
      hi = fmaxf(hi, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w)));
    }
    done = n4 * 4;
  }
  for (size_t i = done + tid; i < n; i += stride) {
    lo = fminf(lo, x[i]);
    hi = fmaxf(hi, x[i]);
  }
  __shared__ float slo[kBlock / dev::kWave], shi[kBlock / dev::kWave];
  lo = dev::wave_min(lo);
  hi = dev::wave_max(hi);
  const int lane = threadIdx.x & 63, wid = threadIdx.x / 64;
  if (lane == 0) {
    slo[wid] = lo;
    shi[wid] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < static_cast<int>(blockDim.x / 64); w++) {
      lo = fminf(lo, slo[w]);
      hi = fmaxf(hi, shi[w]);
    }
    partial[blockIdx.x] = make_float2(lo, hi);
  }
}

__global__ __launch_bounds__(kBlock) void minmax_pass2(const float2 *__restrict__ partial,
                                                       int np, float *__restrict__ out) {
  float lo = partial[0].x, hi = partial[0].y;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    lo = fminf(lo, partial[i].x);
    hi = fmaxf(hi, partial[i].y);
  }
  __shared__ float slo[kBlock / 64], shi[kBlock / 64];
  lo = dev::wave_min(lo);
  hi = dev::wave_max(hi);
  const int lane = threadIdx.x & 63, wid = threadIdx.x / 64;
  if (lane == 0) {
    slo[wid] = lo;
    shi[wid] = hi;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < static_cast<int>(blockDim.x / 64); w++) {
      lo = fminf(lo, slo[w]);
      hi = fmaxf(hi, shi[w]);
    }
    out[0] = lo;
    out[1] = hi;
  }
}

// uint8 plane min/max: blocks walk rows, lanes walk 16-byte column groups
// (one uint4 load per step over the 16-aligned middle of a row; scalar head
// and tail).  4-byte groups ran at 2.2 TB/s on an 8192 x 8192 plane.
__device__ __forceinline__ void mm_word(unsigned v, unsigned &lo, unsigned &hi) {
  const unsigned b0 = v & 255u, b1 = (v >> 8) & 255u, b2 = (v >> 16) & 255u, b3 = v >> 24;
  lo = min(lo, min(min(b0, b1), min(b2, b3)));
  hi = max(hi, max(max(b0, b1), max(b2, b3)));
}

// Planes over grid.y (plane stride `pstride` bytes), partial[plane][block].
__global__ __launch_bounds__(kBlock) void minmax2d_pass1(const uint8_t *__restrict__ src,
                                                         int stride, int64_t pstride, int w,
                                                         int h, uint2 *__restrict__ partial) {
  src += blockIdx.y * pstride;
  partial += static_cast<size_t>(blockIdx.y) * gridDim.x;
  unsigned lo = 255, hi = 0;
  for (int y = blockIdx.x; y < h; y += gridDim.x) {
    const uint8_t *row = src + static_cast<size_t>(y) * stride;
    const int head = static_cast<int>((16 - (reinterpret_cast<uintptr_t>(row) & 15)) & 15);
    const int hcount = head < w ? head : w;
    for (int x = threadIdx.x; x < hcount; x += blockDim.x) {
      lo = min(lo, static_cast<unsigned>(row[x]));
      hi = max(hi, static_cast<unsigned>(row[x]));
    }
    const int nv = (w - hcount) / 16;
    const uint4 *r16 = reinterpret_cast<const uint4 *>(row + hcount);
    for (int i = threadIdx.x; i < nv; i += blockDim.x) {
      const uint4 v = r16[i];
      mm_word(v.x, lo, hi);
      mm_word(v.y, lo, hi);
      mm_word(v.z, lo, hi);
      mm_word(v.w, lo, hi);
    }
    for (int x = hcount + nv * 16 + threadIdx.x; x < w; x += blockDim.x) {
      lo = min(lo, static_cast<unsigned>(row[x]));
      hi = max(hi, static_cast<unsigned>(row[x]));
    }
  }
  __shared__ unsigned slo[kBlock], shi[kBlock];
  slo[threadIdx.x] = lo;
  shi[threadIdx.x] = hi;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (static_cast<int>(threadIdx.x) < s) {
      slo[threadIdx.x] = min(slo[threadIdx.x], slo[threadIdx.x + s]);
      shi[threadIdx.x] = max(shi[threadIdx.x], shi[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = make_uint2(slo[0], shi[0]);
}

__global__ __launch_bounds__(kBlock) void minmax2d_pass2(const uint2 *__restrict__ partial,
                                                         int np, uint8_t *__restrict__ out) {
  partial += static_cast<size_t>(blockIdx.x) * np;  // one block per plane
  out += 2 * blockIdx.x;
  __shared__ unsigned slo[kBlock], shi[kBlock];
  unsigned lo = 255, hi = 0;
  for (int i = threadIdx.x; i < np; i += blockDim.x) {
    lo = min(lo, partial[i].x);
    hi = max(hi, partial[i].y);
  }
  slo[threadIdx.x] = lo;
  shi[threadIdx.x] = hi;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (static_cast<int>(threadIdx.x) < s) {
      slo[threadIdx.x] = min(slo[threadIdx.x], slo[threadIdx.x + s]);
      shi[threadIdx.x] = max(shi[threadIdx.x], shi[threadIdx.x + s]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[0] = static_cast<uint8_t>(slo[0]);
    out[1] = static_cast<uint8_t>(shi[0]);
  }
}

// dst = (src - min) / ((max - min) / 2) - 1, same operation order as the
// scalar reference so results agree to the last bit.  Rows over grid.y;
// each lane converts 4 pixels per step (one uchar4 load, one float4 store:
// the wave's stores stay contiguous) over the 4-aligned middle of a row
// whose destination is 16-byte aligned at the same column, scalar head and
// tail otherwise.  8192 x 8192: one pixel per lane 1.96 TB/s, this 3.9,
// 16 pixels per lane (four float4 stores 64 B apart across the wave) 2.8
// (tools/bench_memops.py, profiles/r2/session6/memops.md).
__device__ __forceinline__ float norm_px(unsigned v, int lo, float diff, bool flat) {
  return flat ? 0.f : (static_cast<int>(v) - lo) / diff - 1.0f;
}

__global__ __launch_bounds__(kBlock) void normalize2d_kernel(
    const uint8_t *__restrict__ src, int sstride, int64_t splane, int w, int h,
    const uint8_t *__restrict__ mm, int vmin, int vmax, float *__restrict__ dst,
    int dstride, int64_t dplane) {
  // planes over grid.z, each with its own {min, max} pair
  src += blockIdx.z * splane;
  dst += blockIdx.z * dplane;
  const int lo = mm ? mm[2 * blockIdx.z] : vmin;
  const int hi = mm ? mm[2 * blockIdx.z + 1] : vmax;
  const bool flat = hi == lo;
  const float diff = (hi - lo) / 2.f;
  const int t0 = blockIdx.x * blockDim.x + threadIdx.x;
  const int ts = gridDim.x * blockDim.x;
  for (int y = blockIdx.y; y < h; y += gridDim.y) {
    const uint8_t *srow = src + static_cast<size_t>(y) * sstride;
    float *drow = dst + static_cast<size_t>(y) * dstride;
    // first column where the source is 4-aligned; vectorise only if the
    // destination is 16-aligned there too
    int head = static_cast<int>((4 - (reinterpret_cast<uintptr_t>(srow) & 3)) & 3);
    if (head > w) head = w;
    const bool vec = (reinterpret_cast<uintptr_t>(drow + head) & 15) == 0;
    if (!vec) head = w;
    for (int x = t0; x < head; x += ts) drow[x] = norm_px(srow[x], lo, diff, flat);
    const int nv = (w - head) / 4;
    const uchar4 *s4 = reinterpret_cast<const uchar4 *>(srow + head);
    float4 *d4 = reinterpret_cast<float4 *>(drow + head);
#pragma unroll 4
    for (int i = t0; i < nv; i += ts) {
      const uchar4 v = s4[i];
      d4[i] = make_float4(norm_px(v.x, lo, diff, flat), norm_px(v.y, lo, diff, flat),
                          norm_px(v.z, lo, diff, flat), norm_px(v.w, lo, diff, flat));
    }
    for (int x = head + 4 * nv + t0; x < w; x += ts) drow[x] = norm_px(srow[x], lo, diff, flat);
  }
}

unsigned partial_count(size_t n) {
  size_t g = (n + kBlock * 4 - 1) / (kBlock * 4);
  if (g > kMaxPartials) g = kMaxPartials;
  if (g == 0) g = 1;
  return static_cast<unsigned>(g);
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" {

vs_status vs_sum(const float *x, size_t n, float *out, vs_stream_t stream) {
  VS_REQUIRE(x && out, "vs_sum: null pointer");
  auto s = static_cast<hipStream_t>(stream);
  if (n == 0) {
    return vs_fill(out, 0.f, 1, stream);  // a kernel, not a memset: the stream may be captured
  }
  const unsigned g = partial_count(n);
  DeviceBuffer part;
  VS_TRY(part.alloc(g * sizeof(float), s));
  hipLaunchKernelGGL(sum_pass1, dim3(g), dim3(kBlock), 0, s, x, n, part.as<float>());
  hipLaunchKernelGGL(sum_pass2, dim3(1), dim3(kBlock), 0, s, part.as<float>(),
                     static_cast<int>(g), out);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_minmax(const float *x, size_t n, float *out, vs_stream_t stream) {
  VS_REQUIRE(x && out && n > 0, "vs_minmax: invalid arguments");
  auto s = static_cast<hipStream_t>(stream);
  const unsigned g = partial_count(n);
  DeviceBuffer part;
  VS_TRY(part.alloc(g * sizeof(float2), s));
  hipLaunchKernelGGL(minmax_pass1, dim3(g), dim3(kBlock), 0, s, x, n,
                     part.as<float2>());
  hipLaunchKernelGGL(minmax_pass2, dim3(1), dim3(kBlock), 0, s,
                     part.as<float2>(), static_cast<int>(g), out);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_minmax2d_u8_batched(const uint8_t *src, int stride, int64_t plane_stride, int w,
                                 int h, int planes, uint8_t *out, vs_stream_t stream) {
  VS_REQUIRE(src && out && w > 0 && h > 0 && stride >= w && planes >= 0,
             "vs_minmax2d_u8: invalid arguments (w=%d h=%d stride=%d planes=%d)", w, h,
             stride, planes);
  VS_REQUIRE(planes <= 1 || plane_stride >= static_cast<int64_t>(stride) * (h - 1) + w,
             "vs_minmax2d_u8: plane stride smaller than a plane");
  if (planes == 0) return VS_OK;
  if (planes > kMaxGridY)
    return batch_chunks(planes, [&](long long p0, int np) {
      return vs_minmax2d_u8_batched(src + p0 * plane_stride, stride, plane_stride, w, h, np,
                                    out + 2 * p0, stream);
    });
  auto s = static_cast<hipStream_t>(stream);
  // blocks per plane: all rows of a lone plane, fewer when many planes
  // already fill the chip
  unsigned g = static_cast<unsigned>(h < static_cast<int>(kMaxPartials) ? h : kMaxPartials);
  const unsigned per_plane = std::max(1u, 16384u / static_cast<unsigned>(planes));
  if (planes > 1 && g > per_plane) g = per_plane;
  DeviceBuffer part;
  VS_TRY(part.alloc(static_cast<size_t>(g) * planes * sizeof(uint2), s));
  hipLaunchKernelGGL(minmax2d_pass1, dim3(g, static_cast<unsigned>(planes)), dim3(kBlock), 0, s,
                     src, stride, plane_stride, w, h, part.as<uint2>());
  hipLaunchKernelGGL(minmax2d_pass2, dim3(static_cast<unsigned>(planes)), dim3(kBlock), 0, s,
                     part.as<uint2>(), static_cast<int>(g), out);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_minmax2d_u8(const uint8_t *src, int stride, int w, int h,
                         uint8_t *out, vs_stream_t stream) {
  return vs_minmax2d_u8_batched(src, stride, 0, w, h, 1, out, stream);
}

vs_status vs_normalize2d_u8_batched(const uint8_t *src, int sstride, int64_t splane, int w,
                                    int h, int planes, const uint8_t *mm, int vmin, int vmax,
                                    float *dst, int dstride, int64_t dplane,
                                    vs_stream_t stream) {
  VS_REQUIRE(src && dst && w > 0 && h > 0 && sstride >= w && dstride >= w && planes >= 0,
             "vs_normalize2d_u8: invalid arguments");
  VS_REQUIRE(mm || vmin <= vmax, "vs_normalize2d_u8: min > max");
  VS_REQUIRE(planes <= 1 || (splane >= static_cast<int64_t>(sstride) * (h - 1) + w &&
                             dplane >= static_cast<int64_t>(dstride) * (h - 1) + w),
             "vs_normalize2d_u8: plane stride smaller than a plane");
  if (planes == 0) return VS_OK;
  if (planes > kMaxGridY)
    return batch_chunks(planes, [&](long long p0, int np) {
      return vs_normalize2d_u8_batched(src + p0 * splane, sstride, splane, w, h, np,
                                       mm ? mm + 2 * p0 : nullptr, vmin, vmax, dst + p0 * dplane,
                                       dstride, dplane, stream);
    });
  // rows over grid.y, the row's 4-pixel groups over grid.x (x blocks only as
  // many as keep ~16 K blocks in flight, so tall images get one per row),
  // planes over grid.z
  unsigned gy = static_cast<unsigned>(h);
  if (gy > 16384) gy = 16384;
  unsigned gx = static_cast<unsigned>((w / 4 + kBlock - 1) / kBlock);
  const unsigned gx_cap = (16384 + gy - 1) / gy;
  if (gx > gx_cap) gx = gx_cap;
  if (gx == 0) gx = 1;
  hipLaunchKernelGGL(normalize2d_kernel, dim3(gx, gy, static_cast<unsigned>(planes)), dim3(kBlock),
                     0, static_cast<hipStream_t>(stream), src, sstride, splane, w, h, mm, vmin,
                     vmax, dst, dstride, dplane);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_normalize2d_u8(const uint8_t *src, int sstride, int w, int h,
                            const uint8_t *mm, int vmin, int vmax, float *dst,
                            int dstride, vs_stream_t stream) {
  return vs_normalize2d_u8_batched(src, sstride, 0, w, h, 1, mm, vmin, vmax, dst, dstride, 0,
                                   stream);
}

}  // extern "C"
