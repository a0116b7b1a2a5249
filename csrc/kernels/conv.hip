// Batched 1D convolution / cross-correlation.
//
// Three algorithms, as in the reference (src/convolve.c), all on the GPU:
//   * direct: LDS-tiled brute force.  A 256-thread block produces 2048
//     consecutive outputs; the filter is walked in 512-tap chunks staged in
//     LDS together with the matching x window (one pad word per 32 so the
//     8-outputs-per-lane sliding window reads are bank-conflict free); each
//     lane keeps a 15-sample register window, i.e. 2 LDS reads per 8 FMAs.
//   * overlap-save: ONE fused kernel for all blocks of all signals.  A
//     workgroup takes two blocks (the first in the real part, the second in
//     the imaginary part of one complex L-point FFT -- valid because the
//     filter is real), transforms them in LDS, multiplies by the filter
//     spectrum in registers, runs the inverse transform with the radix order
//     reversed (no LDS round trip in between, fft_core.h) and writes the
//     `step` valid samples of each block.  The reference runs this block loop
//     serially through FFTF (src/convolve.c:181-228).
//   * FFT: the same fused kernel with a single block per signal when the
//     padded length fits one workgroup (<= 16384); beyond that a four-step
//     transform through HBM (fft.hip) with the spectra multiplied in place.
// Correlation is convolution with the filter reversed at upload
// (src/convolve.c:167-171, :302-306), except in the direct kernel which reads
// the taps reversed.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "csrc/kernels/device.h"
#include "csrc/kernels/fft_core.h"
#include "csrc/kernels/fft_plan.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace conv {
extern thread_local int g_conv_buf, g_conv_real, g_conv_real_all, g_conv_fused4;  // tuning knobs, defined below
namespace {

using fft::cmul;
using fft::Plan;
using fft::reg_index;

// smallest real-block transform (L = 2^kRealMinLog real samples, M = L / 2)
constexpr int kRealMinLog = 7;

// ------------------------------------------------------------- direct
constexpr int kDirThreads = 256;
constexpr int kDirPerThread = 8;
constexpr int kDirOut = kDirThreads * kDirPerThread;  // outputs per block
constexpr int kDirTaps = 512;                          // taps per LDS chunk
constexpr int kDirX = kDirOut + kDirTaps;              // x window (+1 spare)

__device__ __forceinline__ int xpad(int i) { return i + (i >> 5); }

// Each lane holds 8 consecutive outputs; written straight out, a wave's store
// instruction would touch 64 separate 32-byte pieces.  Bounce them through
// the (reused) LDS window so every store instruction writes 256 consecutive
// bytes per wave.  `buf` must hold kDirOut floats.
__device__ __forceinline__ void store_outputs(const float (&acc)[kDirPerThread], float *buf,
                                              float *__restrict__ yrow, int n0, int q0,
                                              int ylen) {
  __syncthreads();  // every lane is done reading the window
#pragma unroll
  for (int r = 0; r < kDirPerThread; r++) buf[q0 + r] = acc[r];
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kDirPerThread; k++) {
    const int i = threadIdx.x + k * kDirThreads;
    // written once, never re-read here: non-temporal (h = 64 direct: 320 -> 437 K
    // Msamples/s at 2^20 x 64, h = 4: 600 -> 662 K; profiles/r3/conv/nt_sites_ab.log)
    if (n0 + i < ylen) __builtin_nontemporal_store(buf[i], yrow + n0 + i);
  }
}

__global__ __launch_bounds__(kDirThreads) void direct_kernel(
    const float *__restrict__ x, int xlen, int64_t xs, const float *__restrict__ h,
    int hlen, int64_t hs, float *__restrict__ y, int64_t ys, int ylen,
    int reverse) {
  __shared__ float sx[kDirX + kDirX / 32 + 1];
  __shared__ float sh[kDirTaps];
  const int sig = blockIdx.y;
  const float *xrow = x + sig * xs;
  const float *hrow = h + sig * hs;
  const int n0 = blockIdx.x * kDirOut;
  const int q0 = threadIdx.x * kDirPerThread;
  float acc[kDirPerThread];
#pragma unroll
  for (int r = 0; r < kDirPerThread; r++) acc[r] = 0.f;

  for (int m0 = 0; m0 < hlen; m0 += kDirTaps) {
    const int taps = min(kDirTaps, hlen - m0);
    __syncthreads();
    for (int i = threadIdx.x; i < kDirTaps; i += kDirThreads) {
      float v = 0.f;
      if (i < taps) v = reverse ? hrow[hlen - 1 - (m0 + i)] : hrow[m0 + i];
      sh[i] = v;
    }
    // x window: xw[i] = x[n0 - m0 - kDirTaps + i], i < kDirX
    const int xbase = n0 - m0 - kDirTaps;
    for (int i = threadIdx.x; i < kDirX; i += kDirThreads) {
      const int p = xbase + i;
      sx[xpad(i)] = (p >= 0 && p < xlen) ? xrow[p] : 0.f;
    }
    __syncthreads();
    // y[n0 + q0 + r] += sum_mm sh[mm] * xw[q0 + r - mm + kDirTaps]
    float w[2 * kDirPerThread];
    const int top = q0 + kDirTaps;
#pragma unroll
    for (int r = 0; r < kDirPerThread; r++) w[kDirPerThread + r] = sx[xpad(top + r)];
    const int tap_end = (taps + kDirPerThread - 1) & ~(kDirPerThread - 1);
    for (int mm = 0; mm < tap_end; mm += kDirPerThread) {
#pragma unroll
      for (int r = 0; r < kDirPerThread; r++)
        w[r] = sx[xpad(top - mm - kDirPerThread + r)];
#pragma unroll
      for (int u = 0; u < kDirPerThread; u++) {
        const float hv = sh[mm + u];
#pragma unroll
        for (int r = 0; r < kDirPerThread; r++)
          acc[r] = fmaf(hv, w[kDirPerThread + r - u], acc[r]);
      }
#pragma unroll
      for (int r = 0; r < kDirPerThread; r++) w[kDirPerThread + r] = w[r];
    }
  }
  store_outputs(acc, sx, y + sig * ys, n0, q0, ylen);
}

// Short filters (h <= HM): taps in registers (zero-padded to HM), the x
// window of the block staged once in LDS, each lane reads its 8 + HM - 1
// window samples with 16-byte LDS reads.  Memory-bound: one pass over x and y.
// VEC (x rows 16-byte aligned): the window starts at n0 - HM, a multiple of
// 4 floats, and is filled with float4 loads; the outputs leave through LDS
// as float4 stores realigned to each row's 16-byte boundaries (the scalar
// build moved 4 bytes per lane per instruction both ways: h = 4 at 3.2 TB/s,
// tools/bench_conv.py HLENS=4).
template <int HM, bool VEC>
__global__ __launch_bounds__(kDirThreads) void direct_small_kernel(
    const float *__restrict__ x, int xlen, int64_t xs, const float *__restrict__ h,
    int hlen, int64_t hs, float *__restrict__ y, int64_t ys, int ylen, int reverse) {
  constexpr int SH = VEC ? 1 : 0;      // window offset of x[n0 - (HM - 1)]
  constexpr int W = kDirOut + HM + 8;  // window floats (+ slack for the b128 reads)
  static_assert(W % 4 == 0, "float4 window");
  __shared__ __attribute__((aligned(16))) float sx[W];
  const int sig = blockIdx.y;
  const float *xrow = x + sig * xs;
  const float *hrow = h + sig * hs;
  const int n0 = blockIdx.x * kDirOut;
  // window: sx[i] = x[n0 - (HM - 1) - SH + i]
  const int xbase = n0 - (HM - 1) - SH;
  if (VEC) {
    for (int i4 = threadIdx.x; i4 < W / 4; i4 += kDirThreads) {
      const int p = xbase + 4 * i4;
      float4 v;
      if (p >= 0 && p + 3 < xlen) {
        v = *reinterpret_cast<const float4 *>(xrow + p);
      } else {
        v.x = (p >= 0 && p < xlen) ? xrow[p] : 0.f;
        v.y = (p + 1 >= 0 && p + 1 < xlen) ? xrow[p + 1] : 0.f;
        v.z = (p + 2 >= 0 && p + 2 < xlen) ? xrow[p + 2] : 0.f;
        v.w = (p + 3 >= 0 && p + 3 < xlen) ? xrow[p + 3] : 0.f;
      }
      reinterpret_cast<float4 *>(sx)[i4] = v;
    }
  } else {
    for (int i = threadIdx.x; i < W; i += kDirThreads) {
      const int p = xbase + i;
      sx[i] = (p >= 0 && p < xlen) ? xrow[p] : 0.f;
    }
  }
  float tap[HM];
#pragma unroll
  for (int m = 0; m < HM; m++)
    tap[m] = m < hlen ? (reverse ? hrow[hlen - 1 - m] : hrow[m]) : 0.f;
  __syncthreads();
  const int q0 = threadIdx.x * kDirPerThread;
  constexpr int NW = (kDirPerThread + HM - 1 + SH + 3) / 4;  // float4 reads per lane
  float w[4 * NW];
#pragma unroll
  for (int c = 0; c < NW; c++) {
    const float4 v = *reinterpret_cast<const float4 *>(sx + q0 + 4 * c);
    w[4 * c] = v.x;
    w[4 * c + 1] = v.y;
    w[4 * c + 2] = v.z;
    w[4 * c + 3] = v.w;
  }
  // y[n0 + q0 + r] = sum_m tap[m] x[n0 + q0 + r - m] = sum_m tap[m] w[r - m + HM - 1 + SH]
  float acc[kDirPerThread];
#pragma unroll
  for (int r = 0; r < kDirPerThread; r++) {
    float a = 0.f;
#pragma unroll
    for (int m = 0; m < HM; m++) a = fmaf(tap[m], w[r - m + HM - 1 + SH], a);
    acc[r] = a;
  }
  float *yrow = y + sig * ys;
  if (VEC) {
    __syncthreads();  // every lane is done reading the window
#pragma unroll
    for (int r = 0; r < kDirPerThread; r++) sx[q0 + r] = acc[r];
    __syncthreads();
    // float4 stores at 16-byte aligned addresses of this row: outputs
    // n0 + d + 4 g (d = the row's misalignment in floats, n0 % 4 == 0); the
    // d leading and 4 - d trailing outputs of the block are stored singly
    const int d = static_cast<int>((4 - ((reinterpret_cast<uintptr_t>(yrow) >> 2) & 3)) & 3);
    constexpr int G = kDirOut / 4;
#pragma unroll
    for (int k = 0; k < kDirPerThread / 4; k++) {
      const int g = threadIdx.x + k * kDirThreads;
      const int o = n0 + d + 4 * g;
      if (d != 0 && g == G - 1) continue;  // reaches into the next block
      const int b = d + 4 * g;
      const float4 v = make_float4(sx[b], sx[b + 1], sx[b + 2], sx[b + 3]);
      if (o + 3 < ylen) {
        typedef float native4 __attribute__((ext_vector_type(4)));
        const native4 nv = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(nv, reinterpret_cast<native4 *>(yrow + o));
      } else {
        if (o < ylen) yrow[o] = v.x;
        if (o + 1 < ylen) yrow[o + 1] = v.y;
        if (o + 2 < ylen) yrow[o + 2] = v.z;
      }
    }
    if (d != 0 && threadIdx.x < 4) {
      // head: outputs n0 .. n0 + d - 1; tail: n0 + kDirOut - 4 + d .. n0 + kDirOut - 1
      const int t = threadIdx.x;
      if (t < d && n0 + t < ylen) yrow[n0 + t] = sx[t];
      const int j = kDirOut - 4 + d + t;
      if (j < kDirOut && n0 + j < ylen) yrow[n0 + j] = sx[j];
    }
  } else {
    store_outputs(acc, sx, yrow, n0, q0, ylen);
  }
}

// Small grids (few signals, short outputs, long filters -- e.g. one
// 512 x 512 convolution, where direct_kernel is a single workgroup doing
// 4096 serial FMAs per lane): 64 outputs per workgroup, the taps split over
// its 8 waves.  The x window and taps are staged into LDS once (every load of
// the fill in flight together), each wave accumulates its tap range with 4
// independent chains, and the 8 partial sums are reduced through LDS.
constexpr int kSplitWaves = 8;
constexpr int kSplitMaxTaps = 4096;

__global__ __launch_bounds__(64 * kSplitWaves) void direct_split_kernel(
    const float *__restrict__ x, int xlen, int64_t xs, const float *__restrict__ h,
    int hlen, int64_t hs, float *__restrict__ y, int64_t ys, int ylen, int reverse) {
  __shared__ float sx[kSplitMaxTaps + 64];
  __shared__ float sh[kSplitMaxTaps];
  __shared__ float part[kSplitWaves][64];
  const int sig = blockIdx.y;
  const float *xrow = x + sig * xs;
  const float *hrow = h + sig * hs;
  const int n0 = blockIdx.x * 64;
  // window: sx[i] = x[n0 - (hlen - 1) + i], i < hlen + 63
  const int xbase = n0 - (hlen - 1);
#pragma unroll 4
  for (int i = threadIdx.x; i < hlen + 63; i += 64 * kSplitWaves) {
    const int p = xbase + i;
    sx[i] = (p >= 0 && p < xlen) ? xrow[p] : 0.f;
  }
#pragma unroll 4
  for (int i = threadIdx.x; i < hlen; i += 64 * kSplitWaves)
    sh[i] = reverse ? hrow[hlen - 1 - i] : hrow[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int per = (hlen + kSplitWaves - 1) / kSplitWaves;
  const int m0 = wave * per, m1 = min(hlen, m0 + per);
  // y[n0 + lane] = sum_m sh[m] * sx[lane + hlen - 1 - m]
  const float *wl = sx + lane + hlen - 1;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int m = m0;
  for (; m + 4 <= m1; m += 4) {
    a0 = fmaf(sh[m], wl[-m], a0);
    a1 = fmaf(sh[m + 1], wl[-m - 1], a1);
    a2 = fmaf(sh[m + 2], wl[-m - 2], a2);
    a3 = fmaf(sh[m + 3], wl[-m - 3], a3);
  }
  for (; m < m1; m++) a0 = fmaf(sh[m], wl[-m], a0);
  part[wave][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (wave == 0 && n0 + lane < ylen) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < kSplitWaves; w++) t += part[w][lane];
    y[sig * ys + n0 + lane] = t;
  }
}

// ------------------------------------------------------ filter spectrum
// hc[f][n] = (reversed?) h[f][n] + 0i for n < hlen, 0 beyond (length L).
__global__ __launch_bounds__(256) void pad_filter_kernel(
    const float *__restrict__ h, int hlen, int64_t hs, int reverse, int logl,
    int nfilt, float2 *__restrict__ hc) {
  const long long L = 1LL << logl;
  const long long total = L * nfilt;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total;
       g += static_cast<long long>(gridDim.x) * 256) {
    const long long f = g >> logl;
    const int n = static_cast<int>(g & (L - 1));
    float v = 0.f;
    if (n < hlen) v = h[f * hs + (reverse ? hlen - 1 - n : n)];
    hc[g] = make_float2(v, 0.f);
  }
}

// ------------------------------------------------ fused block convolution
// Cache policy of the block kernels' output stores (aux operand of the
// buffer stores: bit 1 = non-temporal).  The outputs are written once and
// never re-read by the kernel; kept out of L2 they stop evicting the block
// overlaps, P / Q tables and twiddles the workgroups share: 2^20 x 4096 x 64
// went from 303 to 334 K Msamples/s per call and from 327 to 366 K through a
// plan.  Non-temporal input loads gained 1 % alone and cost 6 % on top of
// the stores (profiles/r3/conv/nt_stores.md).
constexpr int kConvStoreAux = 2;

struct BlockArgs {
  const float *x;
  int64_t xs;
  int xlen;
  float *y;
  int64_t ys;
  int ylen;
  const float2 *H;  // spectrum, natural order, L per filter
  int h_per_signal;
  int pre;    // history samples per block (h_len - 1 for overlap-save)
  int step;   // valid outputs per block
  int nblk;   // block slots per signal (even when filters are per signal)
  long long nslots;
  float scale;
};

// Block pair p = slots 2p and 2p + 1 (the real and imaginary part of one
// complex transform).  Rows of slots that do not exist (past the last
// signal / past the output) are redirected to row 0 so every load address is
// valid; their samples are zeroed and their outputs not stored.
struct PairPos {
  long long sig0, sig1;
  int b0, b1;
  bool ok0, ok1;
};

__device__ __forceinline__ PairPos pair_pos(const BlockArgs &a, long long p) {
  PairPos q;
  const long long s0 = 2 * p, s1 = s0 + 1;
  q.sig0 = s0 / a.nblk;
  q.sig1 = s1 / a.nblk;
  q.b0 = static_cast<int>(s0 - q.sig0 * a.nblk);
  q.b1 = static_cast<int>(s1 - q.sig1 * a.nblk);
  q.ok0 = q.b0 * static_cast<long long>(a.step) < a.ylen;
  q.ok1 = s1 < a.nslots && q.b1 * static_cast<long long>(a.step) < a.ylen;
  return q;
}

// Inputs of the pair in the first pass's register pattern.  BUF: raw buffer
// loads through one descriptor per slot -- the hardware range check returns
// 0 for samples before / past the row and for a slot that does not exist
// (zero records), so the loads need no select and can all be in flight
// before the first butterfly (a select per element made hipcc wait for each
// load group before issuing the next).  !BUF (rows of 2^29 samples or more,
// beyond a 32-bit byte offset): clamped flat loads, zeroed afterwards.
template <class PL, bool BUF>
__device__ __forceinline__ void load_pair(const BlockArgs &a, const PairPos &q, int t,
                                          float2 (&v)[PL::E]) {
  const float *x0 = a.x + (q.ok0 ? q.sig0 : 0) * a.xs;
  const float *x1 = a.x + (q.ok1 ? q.sig1 : 0) * a.xs;
  const int st0 = q.b0 * a.step - a.pre, st1 = q.b1 * a.step - a.pre;
  constexpr int R0 = PL::first_radix(false);
  // buffer loads only from non-negative offsets: the first block of a
  // signal (history before sample 0) takes the flat path
  if (BUF && st0 >= 0 && st1 >= 0) {
    const auto r0 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x0), 0,
                                                      q.ok0 ? 4 * a.xlen : 0, 0x00020000);
    const auto r1 = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(x1), 0,
                                                      q.ok1 ? 4 * a.xlen : 0, 0x00020000);
    const int o0 = 4 * (st0 + t), o1 = 4 * (st1 + t);
#pragma unroll
    for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
      for (int j = 0; j < R0; j++) {
        const int d = 4 * (reg_index<PL, R0>(0, b, j));
        // (the b32 builtins move raw bits: uint32)
        v[b * R0 + j] =
            make_float2(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r0, o0 + d, 0, 0)),
                        __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r1, o1 + d, 0, 0)));
      }
  } else {
    const int last = a.xlen - 1;
#pragma unroll
    for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
      for (int j = 0; j < R0; j++) {
        const int n = reg_index<PL, R0>(t, b, j);
        const int p0 = st0 + n, p1 = st1 + n;
        const float u0 = x0[min(max(p0, 0), last)];
        const float u1 = x1[min(max(p1, 0), last)];
        v[b * R0 + j] =
            make_float2(q.ok0 && static_cast<unsigned>(p0) <= static_cast<unsigned>(last) ? u0 : 0.f,
                        q.ok1 && static_cast<unsigned>(p1) <= static_cast<unsigned>(last) ? u1 : 0.f);
      }
  }
}

// Multiply by the filter spectrum (both slots share it).
template <class PL>
__device__ __forceinline__ void mul_spectrum(const BlockArgs &a, const PairPos &q, int t,
                                             float2 (&v)[PL::E]) {
  const float2 *H = a.H + (a.h_per_signal ? q.sig0 * PL::N : 0);
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++)
      v[b * RL + j] = cmul(v[b * RL + j], H[reg_index<PL, RL>(t, b, j)]);
}

// The `step` valid outputs of each slot, from the inverse transform's last
// pass (the first radix of the forward plan).  BUF: buffer stores whose range
// check drops outputs past the row and every store of a missing slot.
template <class PL, bool BUF>
__device__ __forceinline__ void store_pair(const BlockArgs &a, const PairPos &q, int t,
                                           const float2 (&v)[PL::E]) {
  constexpr int RI = PL::radix(0);
  float *y0 = a.y + (q.ok0 ? q.sig0 : 0) * a.ys;
  float *y1 = a.y + (q.ok1 ? q.sig1 : 0) * a.ys;
  const int base0 = q.b0 * a.step - a.pre, base1 = q.b1 * a.step - a.pre;
  if constexpr (BUF) {
    const auto w0 = __builtin_amdgcn_make_buffer_rsrc(y0, 0, q.ok0 ? 4 * a.ylen : 0, 0x00020000);
    const auto w1 = __builtin_amdgcn_make_buffer_rsrc(y1, 0, q.ok1 ? 4 * a.ylen : 0, 0x00020000);
#pragma unroll
    for (int b = 0; b < PL::E / RI; b++)
#pragma unroll
      for (int j = 0; j < RI; j++) {
        const int n = reg_index<PL, RI>(t, b, j) - a.pre;
        if (n < 0 || n >= a.step) continue;
        const float2 r = v[b * RI + j];
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.x * a.scale), w0,
                                              4 * (base0 + a.pre + n), 0, kConvStoreAux);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.y * a.scale), w1,
                                              4 * (base1 + a.pre + n), 0, kConvStoreAux);
      }
  } else {
#pragma unroll
    for (int b = 0; b < PL::E / RI; b++)
#pragma unroll
      for (int j = 0; j < RI; j++) {
        const int n = reg_index<PL, RI>(t, b, j) - a.pre;
        if (n < 0 || n >= a.step) continue;
        const float2 r = v[b * RI + j];
        const long long o0 = static_cast<long long>(q.b0) * a.step + n;
        const long long o1 = static_cast<long long>(q.b1) * a.step + n;
        if (q.ok0 && o0 < a.ylen) __builtin_nontemporal_store(r.x * a.scale, y0 + o0);
        if (q.ok1 && o1 < a.ylen) __builtin_nontemporal_store(r.y * a.scale, y1 + o1);
      }
  }
}

// One workgroup per block pair.  No barrier between the transforms: the
// forward transform's last LDS read is followed by a barrier inside it.
template <int LOGN, bool BUF>
__global__ __launch_bounds__(Plan<LOGN>::TPS, 1) void block_conv_kernel(
    BlockArgs a, const float2 *__restrict__ tw) {
  using PL = Plan<LOGN>;
  __shared__ float2 lds[PL::kLds];
  const int t = threadIdx.x;
  const PairPos q = pair_pos(a, blockIdx.x);
  float2 v[PL::E];
  load_pair<PL, BUF>(a, q, t, v);
  // every input load in flight before the first butterfly consumes one (the
  // scheduler otherwise splits them into dependent batches)
  __builtin_amdgcn_sched_barrier(0);
  fft::transform<PL, false, false>(v, lds, t, tw);
  mul_spectrum<PL>(a, q, t, v);
  fft::transform<PL, true, true>(v, lds, t, tw);
  store_pair<PL, BUF>(a, q, t, v);
}

// Buffer addressing needs every byte offset of a row in 31 bits.
inline bool buffer_ok(const BlockArgs &a) {
  return g_conv_buf && a.xlen < (1 << 29) && a.ylen < (1 << 29);
}

template <int LOGN>
void launch_block_t(const BlockArgs &a, const float2 *tw, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>((a.nslots + 1) / 2);
  if (buffer_ok(a))
    hipLaunchKernelGGL((block_conv_kernel<LOGN, true>), dim3(grid), dim3(Plan<LOGN>::TPS), 0, s,
                       a, tw);
  else
    hipLaunchKernelGGL((block_conv_kernel<LOGN, false>), dim3(grid), dim3(Plan<LOGN>::TPS), 0, s,
                       a, tw);
}


// Diagnostic build only (make stamps, tools/conv_stamps.py): per-phase
// shader-clock stamps of the real-block kernel; the hooks compile to nothing
// in the shipped library and their code lives in csrc/diag/.
#ifdef VS_CONV_STAMPS
#include "csrc/diag/conv_stamps.inc"
#else
#define VS_STAMP_DECL()
#define VS_STAMP(i)
#define VS_STAMP_FLUSH()
#endif

// --------------------------------------- real-block fused convolution
// One workgroup per block of L = 2M real samples, transformed as an M-point
// complex FFT of z[m] = x[2m] + i x[2m+1].  The real-spectrum split, the
// filter product and the inverse merge are one linear map per bin pair
// (k, M - k):
//   Z'[k] = P[k] Z[k] + Q[k] conj(Z[M - k])        (real_filter_kernel)
// so the spectrum step is one LDS exchange (each thread reads the mirror
// bin of each of its own bins) and two complex products.  An M = 8192
// transform (L = 16384, the overlap-save block of a 4096-tap filter) needs
// 64 KiB of LDS: two workgroups per CU, so one's HBM loads / stores and LDS
// exchanges overlap the other's butterflies -- the pair kernel above keeps a
// 16384-point complex image (128 KiB, one workgroup per CU) and serialises
// them.
struct RealArgs {
  const float *x;
  int64_t xs;
  int xlen;
  float *y;      // this pass's output origin (row 0, sample 0)
  int64_t ys;
  int ylen;      // outputs of this pass per row
  int yroom;     // writable samples from y per row (>= ylen)
  const float4 *PQ;  // {P, Q}, M per filter
  int pq_per_signal;
  int pre;       // history samples per block (taps - 1 for overlap-save)
  int step;      // valid outputs per block
  int nblk;      // blocks per signal
  int accumulate;  // y += result (partitioned long filters)
};

template <class PL, bool BUF>
__device__ __forceinline__ void load_real(const RealArgs &a, const float *xr, int st, int t,
                                          float2 (&v)[PL::E]) {
  constexpr int R0 = PL::first_radix(false);
  if (BUF && st >= 0) {
    // 8-byte buffer loads; the range check zeroes samples past the row
    // (checked per dword: tests/test_convolve.py odd lengths)
    const auto r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(xr), 0, 4 * a.xlen,
                                                     0x00020000);
    const int o = 4 * (st + 2 * t);
#pragma unroll
    for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
      for (int j = 0; j < R0; j++) {
        const int d = 8 * reg_index<PL, R0>(0, b, j);
        const auto w = __builtin_amdgcn_raw_buffer_load_b64(r, o + d, 0, 0);
        v[b * R0 + j] = make_float2(__uint_as_float(w[0]), __uint_as_float(w[1]));
      }
  } else {
    const int last = a.xlen - 1;
#pragma unroll
    for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
      for (int j = 0; j < R0; j++) {
        const int p = st + 2 * reg_index<PL, R0>(t, b, j);
        const float u0 = xr[min(max(p, 0), last)];
        const float u1 = xr[min(max(p + 1, 0), last)];
        v[b * R0 + j] = make_float2(static_cast<unsigned>(p) <= static_cast<unsigned>(last) ? u0 : 0.f,
                                    static_cast<unsigned>(p + 1) <= static_cast<unsigned>(last) ? u1 : 0.f);
      }
  }
}

template <class PL, bool BUF>
__device__ __forceinline__ void store_real(const RealArgs &a, float *yr, int st, int t,
                                           const float2 (&v)[PL::E]) {
  constexpr int R0 = PL::radix(0);  // last pass of the reversed-radix inverse
  // valid block positions [lo, hi): history dropped, row end respected
  const int lo = a.pre, hi = min(a.pre + a.step, a.ylen - st);
  if constexpr (BUF) {
    // The descriptor covers exactly the valid outputs [st + lo, st + hi):
    // history positions get negative offsets (as unsigned: past the range)
    // and are dropped by the buffer unit -- no per-element compares or
    // branches.  lo is even (run_real), so no pair straddles the start; a
    // pair straddling the row end keeps its in-range first dword (range
    // check per dword; tests: odd / even filter and row lengths).
    const auto w = __builtin_amdgcn_make_buffer_rsrc(yr + st + lo, 0, 4 * max(hi - lo, 0),
                                                     0x00020000);
#pragma unroll
    for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
      for (int j = 0; j < R0; j++) {
        const int p = 2 * reg_index<PL, R0>(t, b, j);
        float2 r = v[b * R0 + j];
        const int off = 4 * (p - lo);
        if (a.accumulate) {
          const auto o = __builtin_amdgcn_raw_buffer_load_b64(w, off, 0, 0);
          r.x += __uint_as_float(o[0]);
          r.y += __uint_as_float(o[1]);
        }
        __attribute__((ext_vector_type(2))) unsigned u = {__float_as_uint(r.x),
                                                           __float_as_uint(r.y)};
        __builtin_amdgcn_raw_buffer_store_b64(u, w, off, 0, kConvStoreAux);
      }
  } else {
#pragma unroll
    for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
      for (int j = 0; j < R0; j++) {
        const int p = 2 * reg_index<PL, R0>(t, b, j);
        const float2 r = v[b * R0 + j];
        const bool ok0 = p >= lo && p < hi, ok1 = p + 1 >= lo && p + 1 < hi;
        float *dst = yr + st + p;
        if (ok0) __builtin_nontemporal_store(a.accumulate ? dst[0] + r.x : r.x, dst);
        if (ok1) __builtin_nontemporal_store(a.accumulate ? dst[1] + r.y : r.y, dst + 1);
      }
  }
}

// Spectrum step of real_conv_kernel on elements [C0, C0 + CN) of v (pattern
// reg_index<RL>): Z'[k] = P[k] Z[k] + Q[k] conj(Z[M - k]).
template <class PL, int C0, int CN>
__device__ __forceinline__ void real_spectrum_chunk(float2 (&v)[PL::E], const float2 *lds,
                                                    const float4 (&pq)[CN], int t) {
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int c = 0; c < CN; c++) {
    const int e = C0 + c;
    const int k = reg_index<PL, RL>(t, e / RL, e % RL);
    const float2 zm = lds[fft::slot<PL>((PL::N - k) & (PL::N - 1))];
    v[e] = fft::cadd(cmul(make_float2(pq[c].x, pq[c].y), v[e]),
                     fft::cmulc(make_float2(pq[c].z, pq[c].w), zm));
  }
}

template <class PL, int C0, int CN>
__device__ __forceinline__ void real_pq_load(const float4 *__restrict__ PQ, int t,
                                             float4 (&pq)[CN]) {
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int c = 0; c < CN; c++) {
    const int e = C0 + c;
    pq[c] = PQ[reg_index<PL, RL>(t, e / RL, e % RL)];
  }
}

// Every global load of this kernel is issued ahead of its use: the input
// block and the forward twiddles (RegTw) at entry, the P / Q table in
// chunks one chunk ahead of the products, the inverse twiddles before the
// spectrum exchange -- TableTw / plain indexing waited for each L2 hit
// right before its use (32 serial P / Q round trips per block).
// Waves per SIMD the compiler must allow for (VGPR budget 512 / waves): the
// 16-point M = 8192 plan runs 8 waves per workgroup, so two workgroups per CU
// (16 waves) need <= 128 VGPRs.
template <int LOGM, int EP>
constexpr int real_min_waves() {
  return Plan<LOGM, EP>::TPS >= 512 && Plan<LOGM, EP>::E == 16 ? 4 : 1;
}

template <int LOGM, int EP, bool BUF>
__global__ __launch_bounds__((Plan<LOGM, EP>::TPS), (real_min_waves<LOGM, EP>())) void real_conv_kernel(
    RealArgs a, const float2 *__restrict__ tw) {
  using PL = Plan<LOGM, EP>;
  constexpr int E = PL::E;
  constexpr int CH = E / 4;  // P / Q chunk (elements)
  __shared__ float2 lds[PL::kLds];
  const int t = threadIdx.x;
  // grid = (blocks per signal, signals): both indices stay in SGPRs (a
  // buffer descriptor built from a VALU-divided index turned every load
  // into a waterfall loop)
  const int sig = blockIdx.y;
  const int blk = blockIdx.x;
  const float *xr = a.x + static_cast<long long>(sig) * a.xs;
  float *yr = a.y + static_cast<long long>(sig) * a.ys;
  const int st = blk * a.step - a.pre;
  VS_STAMP_DECL();
  VS_STAMP(0);
  float2 v[E];
  load_real<PL, BUF>(a, xr, st, t, v);
  fft::RegTw<PL, false> twf;
  twf.load(t, tw);
  __builtin_amdgcn_sched_barrier(0);
  VS_STAMP(1);
  fft::transform<PL, false, false>(v, lds, t, twf);
  VS_STAMP(2);
  // v: Z[k], k = reg_index<RL>; the inverse starts from the same pattern
  constexpr int RL = PL::last_radix(false);
  const float4 *PQ = a.PQ + (a.pq_per_signal ? static_cast<long long>(sig) * PL::N : 0);
  float4 pq0[CH], pq1[CH];
  real_pq_load<PL, 0, CH>(PQ, t, pq0);
  fft::RegTw<PL, true> twi;
  twi.load(t, tw);
#pragma unroll
  for (int b = 0; b < E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++)
      lds[fft::slot<PL>(reg_index<PL, RL>(t, b, j))] = v[b * RL + j];
  fft::lds_barrier();
  real_pq_load<PL, CH, CH>(PQ, t, pq1);
  __builtin_amdgcn_sched_barrier(0);
  real_spectrum_chunk<PL, 0, CH>(v, lds, pq0, t);
  real_pq_load<PL, 2 * CH, CH>(PQ, t, pq0);
  __builtin_amdgcn_sched_barrier(0);
  real_spectrum_chunk<PL, CH, CH>(v, lds, pq1, t);
  real_pq_load<PL, 3 * CH, CH>(PQ, t, pq1);
  __builtin_amdgcn_sched_barrier(0);
  real_spectrum_chunk<PL, 2 * CH, CH>(v, lds, pq0, t);
  __builtin_amdgcn_sched_barrier(0);
  real_spectrum_chunk<PL, 3 * CH, CH>(v, lds, pq1, t);
  fft::lds_barrier();
  VS_STAMP(3);
  fft::transform<PL, true, true>(v, lds, t, twi);
  VS_STAMP(4);
  store_real<PL, BUF>(a, yr, st, t, v);
  VS_STAMP_FLUSH();
}

// P, Q of the real-block kernel, one launch per filter straight from the
// taps: the zero-padded (optionally reversed) filter of L = 2M samples as an
// M-point complex transform of its even/odd pairs Zh, then the real split
//   H[k] = a Zh[k] + b conj(Zh[M-k]),  H[M-k] = conj(a) Zh[M-k] + conj(b) conj(Zh[k])
// and the fold
//   a = (1 - i W^k)/2, b = (1 + i W^k)/2   (split:  X[k] = a Z[k] + b Z*[M-k])
//   c = conj(a), d = conj(b)               (merge:  Z'[k] = c Y[k] + d Y*[M-k])
//   P = (c a H[k] + d b H*[M-k]) / M,  Q = (c b H[k] + d a H*[M-k]) / M
// with W = exp(-2 pi i / L) (k = 0 pairs with itself: H[M] is the Nyquist bin).
// One workgroup per filter, 16 points per thread whatever plan the block
// kernel uses (a lone workgroup is latency-bound: more waves, and every
// global load -- taps, both twiddle sets, the W^k of the split -- issued
// before the first butterfly).
template <int LOGM>
__global__ __launch_bounds__((Plan<LOGM>::TPS)) void real_filter_kernel(
    const float *__restrict__ h, int hlen, int64_t hs, int reverse, int part_taps,
    const float2 *__restrict__ tw, const float2 *__restrict__ twl, float4 *__restrict__ PQ) {
  using PL = Plan<LOGM>;
  constexpr int E = PL::E;
  __shared__ float2 lds[PL::kLds];
  const int t = threadIdx.x;
  // grid = (partitions of part_taps taps, filters): partition p holds taps
  // [p part_taps, (p + 1) part_taps) of the (reversed) filter
  const float *hr = h + static_cast<long long>(blockIdx.y) * hs;
  const int p0 = static_cast<int>(blockIdx.x) * part_taps;
  const int taps = min(part_taps, hlen - p0);
  constexpr int R0 = PL::first_radix(false);
  constexpr int RL = PL::last_radix(false);
  float2 v[E], wk[E];
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int n = 2 * reg_index<PL, R0>(t, e / R0, e % R0);
    const int g = p0 + n;  // tap index in the (reversed) filter
    const int i0 = reverse ? hlen - 1 - g : g, i1 = reverse ? hlen - 2 - g : g + 1;
    const float u0 = hr[n < taps ? i0 : 0], u1 = hr[n + 1 < taps ? i1 : 0];
    v[e] = make_float2(n < taps ? u0 : 0.f, n + 1 < taps ? u1 : 0.f);
  }
#pragma unroll
  for (int e = 0; e < E; e++) wk[e] = twl[reg_index<PL, RL>(t, e / RL, e % RL)];
  fft::RegTw<PL, false> twf;
  twf.load(t, tw);
  __builtin_amdgcn_sched_barrier(0);
  fft::transform<PL, false, false>(v, lds, t, twf);
#pragma unroll
  for (int e = 0; e < E; e++) lds[fft::slot<PL>(reg_index<PL, RL>(t, e / RL, e % RL))] = v[e];
  fft::lds_barrier();
  float4 *out = PQ + (static_cast<long long>(blockIdx.y) * gridDim.x + blockIdx.x) * PL::N;
  const float sc = 1.0f / static_cast<float>(PL::N);
#pragma unroll
  for (int e = 0; e < E; e++) {
    const int k = reg_index<PL, RL>(t, e / RL, e % RL);
    const float2 zk = v[e];
    const float2 zm = lds[fft::slot<PL>((PL::N - k) & (PL::N - 1))];
    const float2 w = wk[e];                    // W^k, W = exp(-2 pi i / L)
    const float2 iw = make_float2(-w.y, w.x);  // i W^k
    const float2 ca = make_float2(0.5f * (1.f - iw.x), -0.5f * iw.y);
    const float2 cb = make_float2(0.5f * (1.f + iw.x), 0.5f * iw.y);
    const float2 zmc = make_float2(zm.x, -zm.y);
    const float2 hk = fft::cadd(cmul(ca, zk), cmul(cb, zmc));
    // conj(H[M-k]) = a conj(Zh[M-k]) + b Zh[k]
    const float2 hm = fft::cadd(cmul(ca, zmc), cmul(cb, zk));
    const float2 cc = make_float2(ca.x, -ca.y);  // (1 + i W^-k)/2 = conj(a)
    const float2 cd = make_float2(cb.x, -cb.y);  // (1 - i W^-k)/2 = conj(b)
    const float2 P = fft::cadd(cmul(cmul(cc, ca), hk), cmul(cmul(cd, cb), hm));
    const float2 Q = fft::cadd(cmul(cmul(cc, cb), hk), cmul(cmul(cd, ca), hm));
    out[k] = make_float4(sc * P.x, sc * P.y, sc * Q.x, sc * Q.y);
  }
}

// P / Q of nfilt filters (stride hs) for the L = 2^(LOGM+1) real block into
// `pq`: per filter, one table of PL::N float4 for each partition of
// part_taps taps (a filter that fits one block: part_taps = hlen).
template <int LOGM>
vs_status launch_real_filter(int correlate, const float *h, int hlen, int64_t hs, int nfilt,
                             float4 *pq, hipStream_t s, int part_taps = 0) {
  vs_status st;
  const float2 *tw = fft::twiddles(LOGM, &st);
  if (!tw) return st;
  const float2 *twl = fft::twiddles(LOGM + 1, &st);
  if (!twl) return st;
  if (part_taps <= 0) part_taps = hlen;
  const unsigned parts = static_cast<unsigned>((hlen + part_taps - 1) / part_taps);
  hipLaunchKernelGGL((real_filter_kernel<LOGM>), dim3(parts, static_cast<unsigned>(nfilt)),
                     dim3(Plan<LOGM>::TPS), 0, s, h, hlen, hs, correlate, part_taps, tw, twl, pq);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// One real-block convolution pass: the filter spectra (unless `pq_pre`
// already holds them -- a vs_conv1d plan) then the block kernel.
template <int LOGM, int EP>
vs_status run_real_t(int correlate, const float *h, int hlen, int64_t hs, int nfilt,
                     RealArgs a, long long nblocks, const float4 *pq_pre, hipStream_t s) {
  using PL = Plan<LOGM, EP>;
  vs_status st;
  const float2 *tw = fft::twiddles(LOGM, &st);
  if (!tw) return st;
  DeviceBuffer pq;
  if (pq_pre) {
    a.PQ = pq_pre;
  } else {
    VS_TRY(pq.alloc(sizeof(float4) * PL::N * static_cast<size_t>(nfilt), s));
    VS_TRY(launch_real_filter<LOGM>(correlate, h, hlen, hs, nfilt, pq.as<float4>(), s));
    a.PQ = pq.as<float4>();
  }
  const dim3 grid(static_cast<unsigned>(a.nblk), static_cast<unsigned>(nblocks / a.nblk));
  if (g_conv_buf && a.xlen < (1 << 29) && a.yroom < (1 << 29))
    hipLaunchKernelGGL((real_conv_kernel<LOGM, EP, true>), grid, dim3(PL::TPS), 0, s, a, tw);
  else
    hipLaunchKernelGGL((real_conv_kernel<LOGM, EP, false>), grid, dim3(PL::TPS), 0, s, a, tw);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// ------------------------- uniformly partitioned overlap-save (long filters)
// Filters longer than one overlap-save block (reference src/convolve.c:116-121
// sizes one block from the filter; :181-228 is its block loop): the filter is
// cut into partitions of B = L / 2 taps and the signal into blocks of L
// samples every B (frequency-domain delay line).  Each signal block is
// transformed once (fdl_forward_kernel: its packed M = B point spectrum Z_s
// goes to memory), the products are accumulated in the spectral domain,
//   Y_b[k] = sum_p P_p[k] Z_{b-p}[k] + Q_p[k] conj(Z_{b-p}[M - k]),
// with the partitions' P / Q tables of the real-block kernel
// (fdl_mac_kernel), and each output block takes one inverse transform
// (fdl_inverse_kernel) -- against one forward and one inverse transform per
// block and partition when every partition runs its own overlap-save pass.
template <int LOGM, int EP, bool BUF>
__global__ __launch_bounds__((Plan<LOGM, EP>::TPS), (real_min_waves<LOGM, EP>())) void fdl_forward_kernel(
    RealArgs a, float2 *__restrict__ Z, const float2 *__restrict__ tw) {
  using PL = Plan<LOGM, EP>;
  constexpr int E = PL::E;
  __shared__ float2 lds[PL::kLds];
  const int t = threadIdx.x;
  const int sig = blockIdx.y;
  const int blk = blockIdx.x;
  const float *xr = a.x + static_cast<long long>(sig) * a.xs;
  const int st = blk * a.step - a.pre;
  float2 v[E];
  load_real<PL, BUF>(a, xr, st, t, v);
  fft::RegTw<PL, false> twf;
  twf.load(t, tw);
  __builtin_amdgcn_sched_barrier(0);
  fft::transform<PL, false, false>(v, lds, t, twf);
  constexpr int RL = PL::last_radix(false);
  float2 *z = Z + (static_cast<long long>(sig) * gridDim.x + blk) * PL::N;
#pragma unroll
  for (int b = 0; b < E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++) {
      typedef float native2 __attribute__((ext_vector_type(2)));
      const native2 nv = {v[b * RL + j].x, v[b * RL + j].y};
      __builtin_nontemporal_store(nv, reinterpret_cast<native2 *>(z + reg_index<PL, RL>(t, b, j)));
    }
}

template <int LOGM, int EP, bool BUF>
__global__ __launch_bounds__((Plan<LOGM, EP>::TPS), (real_min_waves<LOGM, EP>())) void fdl_inverse_kernel(
    RealArgs a, const float2 *__restrict__ Y, const float2 *__restrict__ tw) {
  using PL = Plan<LOGM, EP>;
  constexpr int E = PL::E;
  __shared__ float2 lds[PL::kLds];
  const int t = threadIdx.x;
  const int sig = blockIdx.y;
  const int blk = blockIdx.x;
  float *yr = a.y + static_cast<long long>(sig) * a.ys;
  const int st = blk * a.step - a.pre;
  constexpr int RL = PL::last_radix(false);
  const float2 *ys = Y + (static_cast<long long>(sig) * gridDim.x + blk) * PL::N;
  float2 v[E];
#pragma unroll
  for (int b = 0; b < E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++) {
      typedef float native2 __attribute__((ext_vector_type(2)));
      const native2 nv = __builtin_nontemporal_load(
          reinterpret_cast<const native2 *>(ys + reg_index<PL, RL>(t, b, j)));
      v[b * RL + j] = make_float2(nv.x, nv.y);
    }
  fft::RegTw<PL, true> twi;
  twi.load(t, tw);
  __builtin_amdgcn_sched_barrier(0);
  fft::transform<PL, true, true>(v, lds, t, twi);
  store_real<PL, BUF>(a, yr, st, t, v);
}

// Spectral accumulation.  One lane owns the bin pair (k, M - k) of kFdlTile
// consecutive output blocks of one signal: 2 kFdlTile accumulators.  The
// partitions go by in groups of kFdlGroup whose P / Q (2 float4 each) stay in
// registers while the lane walks the source blocks the group needs, so
// every Z load (16 bytes) feeds up to 4 kFdlGroup complex multiply-adds.
// Groups of 4: 0.38 / 0.94 ms for 8 / 25 partitions at 2^20 x 64 (about
// 5 TB/s of Z reads and Y writes); groups of 8 read less but run at two waves
// per SIMD and lose 7-14 % (profiles/r3/conv/fdl.md).  Kept as the A/B arm of
// the LDS-staged kernel below (vs_tune_set("fdl_mac_lds", 0)).
constexpr int kFdlTile = 16;
constexpr int kFdlGroup = 4;

// acc += P z + Q conj(zc), pq = (P.re, P.im, Q.re, Q.im): eight fused
// multiply-adds straight into the accumulator.
__device__ __forceinline__ void fdl_acc(float2 &acc, const float4 pq, const float2 z,
                                        const float2 zc) {
  acc.x = fmaf(pq.x, z.x, acc.x);
  acc.y = fmaf(pq.x, z.y, acc.y);
  acc.x = fmaf(-pq.y, z.y, acc.x);
  acc.y = fmaf(pq.y, z.x, acc.y);
  acc.x = fmaf(pq.z, zc.x, acc.x);
  acc.y = fmaf(pq.w, zc.x, acc.y);
  acc.x = fmaf(pq.w, zc.y, acc.x);
  acc.y = fmaf(-pq.z, zc.y, acc.y);
}

struct FdlMac {
  const float2 *Z;   // [batch][nsrc][M]
  const float4 *PQ;  // [filters][parts][M]
  float2 *Y;         // [batch][nblk][M]
  int nsrc, nblk, parts, m, pq_per_signal;
};

__global__ __launch_bounds__(256) void fdl_mac_kernel(FdlMac a) {
  constexpr int G = kFdlGroup;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j > a.m / 2) return;
  const int k = j, km = (a.m - j) & (a.m - 1);
  const long long sig = blockIdx.z;
  const int b0 = blockIdx.y * kFdlTile;
  const float2 *Z = a.Z + sig * a.nsrc * a.m;
  const float4 *PQ = a.PQ + (a.pq_per_signal ? sig * a.parts * a.m : 0);
  float2 acck[kFdlTile], accm[kFdlTile];
#pragma unroll
  for (int i = 0; i < kFdlTile; i++) acck[i] = accm[i] = make_float2(0.f, 0.f);
  for (int pc = 0; pc < a.parts; pc += G) {
    float4 pk[G], pm[G];
#pragma unroll
    for (int pp = 0; pp < G; pp++) {
      pk[pp] = pm[pp] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (pc + pp < a.parts) {
        pk[pp] = PQ[static_cast<long long>(pc + pp) * a.m + k];
        pm[pp] = PQ[static_cast<long long>(pc + pp) * a.m + km];
      }
    }
#pragma unroll
    for (int i = 0; i < kFdlTile + G - 1; i++) {
      // source block s feeds output b0 + i - (G - 1) + pp through partition pc + pp
      const int s = b0 - pc - (G - 1) + i;
      if (s < 0 || s >= a.nsrc) continue;
      const float2 zk = Z[static_cast<long long>(s) * a.m + k];
      const float2 zm = Z[static_cast<long long>(s) * a.m + km];
#pragma unroll
      for (int pp = 0; pp < G; pp++) {
        const int o = i - (G - 1) + pp;
        if (o < 0 || o >= kFdlTile) continue;
        fdl_acc(acck[o], pk[pp], zk, zm);
        fdl_acc(accm[o], pm[pp], zm, zk);
      }
    }
  }
  float2 *Y = a.Y + sig * a.nblk * a.m;
#pragma unroll
  for (int o = 0; o < kFdlTile; o++) {
    if (b0 + o >= a.nblk) break;
    typedef float native2 __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(native2{acck[o].x, acck[o].y},
                                reinterpret_cast<native2 *>(Y + static_cast<long long>(b0 + o) * a.m + k));
    __builtin_nontemporal_store(native2{accm[o].x, accm[o].y},
                                reinterpret_cast<native2 *>(Y + static_cast<long long>(b0 + o) * a.m + km));
  }
}

// Spectral accumulation with the source spectra staged in LDS.  A workgroup
// owns 64 bin pairs (k, M - k) of kFdlLdsTile consecutive output blocks of one
// signal and walks the partitions in chunks of at most `pc_max`: the
// kFdlLdsTile + chunk - 1 source blocks a chunk needs are read from memory
// once into LDS (1 KiB per block), each wave accumulates kFdlLdsTile / 4
// outputs, and a partition's P / Q pair is loaded once per wave for all of
// them.  Against the register kernel above Z is read (tile + parts - 1) / tile
// times instead of 1.19 times per group of 4 partitions.
constexpr int kFdlLdsTile = 32;
constexpr int kFdlLdsBins = 64;
constexpr int kFdlLdsChunk = 32;  // (32 + 32 - 1) KiB of LDS, under the 64 KiB dynamic limit

template <int PCMAX>
__global__ __launch_bounds__(256, (PCMAX > 16 ? 2 : 3)) void fdl_mac_lds_kernel(FdlMac a) {
  constexpr int pc_max = PCMAX;
  extern __shared__ float2 zl[];  // [rows][128]: 64 bins k, then their 64 mirrors
  constexpr int NB = kFdlLdsBins, OPT = kFdlLdsTile / 4;
  const int t = threadIdx.x, jj = t & (NB - 1), sub = t >> 6;
  const int half = a.m / 2, mask = a.m - 1;
  const int j = blockIdx.x * NB + jj;
  const bool live = j <= half;
  const int k = live ? j : 0, km = live ? (a.m - j) & mask : 0;
  const long long sig = blockIdx.z;
  const int b0 = blockIdx.y * kFdlLdsTile;
  const float2 *Z = a.Z + sig * a.nsrc * a.m;
  const float4 *PQ = a.PQ + (a.pq_per_signal ? sig * a.parts * a.m : 0);
  float2 acck[OPT], accm[OPT];
#pragma unroll
  for (int i = 0; i < OPT; i++) acck[i] = accm[i] = make_float2(0.f, 0.f);
  for (int pc0 = 0; pc0 < a.parts; pc0 += pc_max) {
    const int pcn = min(pc_max, a.parts - pc0);
    const int rows = kFdlLdsTile + pcn - 1;
    const int s0 = b0 - pc0 - (pcn - 1);  // row r holds source block s0 + r
    if (pc0) __syncthreads();             // the previous chunk's readers are done
    // every load of the chunk in flight before the first LDS store
    constexpr int kLoads = (kFdlLdsTile + PCMAX - 1 + 1) / 2;  // two rows per pass of 256 lanes
    float2 v[kLoads];
    const int c = t & (2 * NB - 1);
    const int jb = blockIdx.x * NB + (c & (NB - 1));
    const int bin = c < NB ? jb : (a.m - jb) & mask;
#pragma unroll
    for (int u = 0; u < kLoads; u++) {
      const int r = 2 * u + (t >> 7);
      const int s = s0 + r;
      v[u] = make_float2(0.f, 0.f);
      if (r < rows && s >= 0 && s < a.nsrc && jb <= half) v[u] = Z[static_cast<long long>(s) * a.m + bin];
    }
#pragma unroll
    for (int u = 0; u < kLoads; u++) {
      const int r = 2 * u + (t >> 7);
      if (r < rows) zl[r * 2 * NB + c] = v[u];
    }
    __syncthreads();
#pragma unroll 2
    for (int p = 0; p < pcn; p++) {
      const float4 pk = PQ[static_cast<long long>(pc0 + p) * a.m + k];
      const float4 pm = PQ[static_cast<long long>(pc0 + p) * a.m + km];
#pragma unroll
      for (int i = 0; i < OPT; i++) {
        // output b0 + o through partition pc0 + p reads source b0 + o - pc0 - p
        const int r = sub * OPT + i - p + (pcn - 1);
        const float2 zk = zl[r * 2 * NB + jj], zm = zl[r * 2 * NB + NB + jj];
        fdl_acc(acck[i], pk, zk, zm);
        fdl_acc(accm[i], pm, zm, zk);
      }
    }
  }
  if (!live) return;
  float2 *Y = a.Y + sig * a.nblk * a.m;
#pragma unroll
  for (int i = 0; i < OPT; i++) {
    const int o = b0 + sub * OPT + i;
    if (o >= a.nblk) break;
    typedef float native2 __attribute__((ext_vector_type(2)));
    __builtin_nontemporal_store(native2{acck[i].x, acck[i].y},
                                reinterpret_cast<native2 *>(Y + static_cast<long long>(o) * a.m + k));
    __builtin_nontemporal_store(native2{accm[i].x, accm[i].y},
                                reinterpret_cast<native2 *>(Y + static_cast<long long>(o) * a.m + km));
  }
}

// 0: register kernel (fdl_mac_kernel), 1: LDS-staged kernel.  vs_tune_set("fdl_mac_lds").
thread_local int g_fdl_mac_lds = 1;
// Partitions per LDS chunk: 0 = by partition count, or 8 / 16 / 32.  vs_tune_set("fdl_mac_chunk").
thread_local int g_fdl_mac_chunk = 0;

// ------------------------------------------ large FFT path (four-step)
// z[p][n] = x[2p][n] + i x[2p+1][n] (zero padded to 2^logm)
__global__ __launch_bounds__(256) void pack_pairs_kernel(
    const float *__restrict__ x, int xlen, int64_t xs, int batch, int logm,
    long long npairs, float2 *__restrict__ z) {
  const long long M = 1LL << logm;
  const long long total = npairs * M;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total;
       g += static_cast<long long>(gridDim.x) * 256) {
    const long long p = g >> logm;
    const int n = static_cast<int>(g & (M - 1));
    const long long s0 = 2 * p, s1 = 2 * p + 1;
    const float a = n < xlen ? x[s0 * xs + n] : 0.f;
    const float b = (n < xlen && s1 < batch) ? x[s1 * xs + n] : 0.f;
    z[g] = make_float2(a, b);
  }
}

__global__ __launch_bounds__(256) void unpack_pairs_kernel(
    const float2 *__restrict__ z, int logm, long long npairs, int batch,
    float *__restrict__ y, int64_t ys, int ylen, float scale) {
  const long long M = 1LL << logm;
  const long long total = npairs * ylen;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total;
       g += static_cast<long long>(gridDim.x) * 256) {
    const long long p = g / ylen;
    const int n = static_cast<int>(g % ylen);
    const float2 v = z[p * M + n];
    y[2 * p * ys + n] = v.x * scale;
    if (2 * p + 1 < batch) y[(2 * p + 1) * ys + n] = v.y * scale;
  }
}

// z[p] *= H[p or 0] over the four-step (permuted) spectrum layout
__global__ __launch_bounds__(256) void spectrum_mul_kernel(
    float2 *__restrict__ z, const float2 *__restrict__ H, int logm,
    long long npairs, int h_per_pair) {
  const long long M = 1LL << logm;
  const long long total = npairs * M;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total;
       g += static_cast<long long>(gridDim.x) * 256) {
    const long long hi = h_per_pair ? g : (g & (M - 1));
    z[g] = cmul(z[g], H[hi]);
  }
}

}  // namespace

// The tuning knobs are per thread (vs_tune_set changes the calling thread's
// values only; vs_tune_reset restores the defaults): concurrent callers never
// see each other's settings, and a plan records what it was built with.
// Tuning knob (vs_tune_set("os_block_log_max", n)): cap of the overlap-save
// block size, for A/B measurements.  The real-block kernel reaches one more
// power of two than the complex transforms (L = 2M real samples).
thread_local int g_os_log_max = fft::kMaxLdsLog + 1;
// Tuning knob (vs_tune_set("os_block_extra", 0/2/3/4)): overlap-save block
// L = 2^(floor(log2 h) + extra); the reference uses 2 (src/convolve.c:116-121).
// 0 (default): 3 while that keeps L <= 8192, else 2 -- the M <= 4096 real
// kernels run ~1.25x more block points per second than the M = 8192 one
// (x = 2^20 x 64, Msamples/s, profiles/r2/conv_block_rule.md):
//   h = 700: 344 -> 388 K, 1000: 260 -> 336 K, 2000: 270 -> 330 K;
//   h = 3000 / 4096 keep L = 8192 / 16384 (L = 16384 / 32768: -7 % / -14 %).
thread_local int g_os_extra = 0;
// Tuning knob (vs_tune_set("conv_fused4", 0/1)): fused three-pass four-step
// FFT convolution (fft::conv_four_step) vs the seven-pass sequence.
thread_local int g_conv_fused4 = 1;
// Tuning knob (vs_tune_set("conv_buffer", 0/1)): buffer-descriptor loads and
// stores in the fused block kernels.
thread_local int g_conv_buf = 1;
// Tuning knob (vs_tune_set("conv_real", 0/1)): real-block kernel for the
// overlap-save / single-block paths (0: pair kernel).
thread_local int g_conv_real = 1;
// Tuning knob (vs_tune_set("conv_real_all", 0/1)): real-block kernel for
// every block size (default: L >= 8192 only, see use_real).
thread_local int g_conv_real_all = 0;

bool use_real(int logl);
int fdl_block_log(int hlen);
int fdl_part_taps(int hlen);
constexpr int kFdlMaxParts = 20;

// Longest row one kernel launch sequence handles: the buffer-descriptor
// loads and stores of the block kernels need every byte offset of a row in
// 31 bits (rows below 2^29 samples).  vs_conv1d cuts longer rows into pieces
// of 2^28 outputs.
// vs_tune_set("conv_piece_log", n) lowers the piece size (tests of the piece
// logic on short rows).
thread_local int g_piece_log = 28;
inline long long piece_out() { return 1LL << g_piece_log; }
inline long long max_call_out() { return 2 * piece_out() - 1; }

// Largest single-workgroup block: the real-block kernel transforms L = 2M
// real samples as an M-point complex FFT, so it reaches 2^(kMaxLdsLog + 1).
int max_block_log() { return use_real(fft::kMaxLdsLog + 1) ? fft::kMaxLdsLog + 1 : fft::kMaxLdsLog; }

int os_block_log(int hlen) {
  // Reference block size 2^(floor(log2 M) + 2) (src/convolve.c:116-121),
  // raised to >= 2048 so every block amortises its transform over >= ~75%
  // useful outputs, capped at the single-workgroup LDS transform.
  int lg = g_os_extra ? g_os_extra : 3;
  int m = hlen;
  while (m >>= 1) lg++;
  if (g_os_extra == 0 && lg > 13) lg--;
  if (lg < 11) lg = 11;
  const int cap = std::min(g_os_log_max, max_block_log());
  if (lg > cap) lg = cap;
  while ((1 << lg) <= hlen && lg < cap) lg++;  // must exceed h - 1
  return lg;
}

// Overlap-save with one block per filter while >= 28 % of each block is
// useful output: the block rule keeps >= 75 % up to h = 8192; past that
// L = 32768 real blocks run ~370 M block points/s at 2^20 x 64 (h = 20000,
// 39 % useful: 144 Gsamples/s; ~104 at 28 %) against ~104 for three or four filter
// partitions of the uniformly partitioned path and 70 for the whole-signal
// four-step FFT (profiles/r2/conv/conv_long.log, profiles/r3/conv/fdl.md).
bool os_single_block(int hlen) {
  const int los = os_block_log(hlen);
  return (1 << los) > hlen - 1 + 16 &&
         static_cast<long long>((1 << los) - (hlen - 1)) * 100 >= 28LL * (1 << los);
}

int select(int64_t xlen, int hlen, int batch) {
  const long long ylen = static_cast<long long>(xlen) + hlen - 1;
  (void)batch;
  // rows cut into pieces (vs_conv1d): no single transform covers them
  if (ylen > max_call_out()) return hlen <= 8 ? VS_CONV_DIRECT : VS_CONV_OVERLAP_SAVE;
  // Direct only for very short filters or signals: at x = 2^20 x 64 the
  // float4 direct kernel runs h <= 8 at ~650 Gsamples/s against ~490 for
  // overlap-save; at h = 16 they are level (505 vs 500 with 16-byte aligned
  // rows, 330 without) and from h = 32 overlap-save wins (490 vs 350)
  // (profiles/r2/session6/conv_small.md).
  if (ylen <= 64 || hlen <= 8 || (hlen <= 32 && xlen < 4096)) return VS_CONV_DIRECT;
  const int los = os_block_log(hlen);
  const bool os_ok = os_single_block(hlen);
  int lm = 1;
  while ((1LL << lm) < ylen) lm++;
  if (lm <= max_block_log() && (!os_ok || ylen <= (1LL << los)))
    return VS_CONV_FFT;  // one block covers the whole output
  if (os_ok) return VS_CONV_OVERLAP_SAVE;
  // Long filter: uniformly partitioned overlap-save up to kFdlMaxParts
  // partitions (its spectral accumulation grows with the partition count:
  // at 2^20 x 64, 8 partitions run 100 Gsamples/s, 13 run 93, 20 run 73, 25
  // run 66, the fused four-step transform 70 whatever the filter), else one
  // padded transform
  // while it exists (vs_conv1d never fails for a valid shape).
  const int parts = (hlen + fdl_part_taps(hlen) - 1) / fdl_part_taps(hlen);
  // L = 32768 blocks (filters past 20 partitions of 8192 taps): 13 partitions run 72
  // Gsamples/s, 25 run 55
  const int max_parts = fdl_block_log(hlen) == 15 ? 14 : kFdlMaxParts;
  return parts <= max_parts || lm > fft::kMaxLog ? VS_CONV_OVERLAP_SAVE : VS_CONV_FFT;
}

// Every run_* entry writes the first `ylen` outputs (<= xlen + hlen - 1) of
// each row: callers that cut a long signal into pieces drop the tail that
// the next piece owns.
vs_status run_direct(int correlate, const float *x, int xlen, int64_t xs,
                     const float *h, int hlen, int64_t hs, float *y, int64_t ys, int ylen,
                     int batch, hipStream_t s) {
  const dim3 grid(static_cast<unsigned>((ylen + kDirOut - 1) / kDirOut),
                  static_cast<unsigned>(batch));
  // VEC: x rows 16-byte aligned (float4 window loads); y rows may start
  // anywhere (the store path realigns per row)
  const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(y) & 3) == 0 && (batch == 1 || xs % 4 == 0);
#define VS_DIRECT_SMALL(HM)                                                               \
  {                                                                                       \
    if (vec)                                                                              \
      hipLaunchKernelGGL((direct_small_kernel<HM, true>), grid, dim3(kDirThreads), 0, s, x, \
                         xlen, xs, h, hlen, hs, y, ys, ylen, correlate);                 \
    else                                                                                  \
      hipLaunchKernelGGL((direct_small_kernel<HM, false>), grid, dim3(kDirThreads), 0, s, \
                         x, xlen, xs, h, hlen, hs, y, ys, ylen, correlate);              \
  }
  if (hlen <= 8) VS_DIRECT_SMALL(8)
  else if (hlen <= 16) VS_DIRECT_SMALL(16)
  else if (hlen <= 32) VS_DIRECT_SMALL(32)
#undef VS_DIRECT_SMALL
  else if (hlen <= kSplitMaxTaps &&
           static_cast<int64_t>(grid.x) * batch < 2 * device_cu_count())
    hipLaunchKernelGGL(direct_split_kernel, dim3((ylen + 63) / 64, batch),
                       dim3(64 * kSplitWaves), 0, s, x, xlen, xs, h, hlen, hs, y, ys, ylen,
                       correlate);
  else
    hipLaunchKernelGGL(direct_kernel, grid, dim3(kDirThreads), 0, s, x, xlen, xs, h,
                       hlen, hs, y, ys, ylen, correlate);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// Spectra (natural order, 2^logl points) of the nfilt filters.
vs_status filter_spectra(int correlate, const float *h, int hlen, int64_t hs,
                         int nfilt, int logl, DeviceBuffer &out, hipStream_t s) {
  const size_t n = (static_cast<size_t>(1) << logl) * nfilt;
  VS_TRY(out.alloc(n * sizeof(float2), s));
  hipLaunchKernelGGL(pad_filter_kernel, dim3(elementwise_grid(n, 256)), dim3(256), 0,
                     s, h, hlen, hs, correlate, logl, nfilt, out.as<float2>());
  VS_HIP(hipGetLastError());
  return fft::launch_c2c_lds(logl, false, out.as<float2>(), out.as<float2>(), nfilt, s);
}

vs_status run_block(int correlate, bool overlap_save, const float *x, int xlen,
                    int64_t xs, const float *h, int hlen, int64_t hs, float *y,
                    int64_t ys, int ylen, int batch, hipStream_t s) {
  int logl;
  if (overlap_save) {
    logl = os_block_log(hlen);
  } else {
    logl = 4;  // smallest instantiated transform
    while ((1 << logl) < xlen + hlen - 1) logl++;
  }
  VS_REQUIRE(logl <= fft::kMaxLdsLog, "block convolution: block 2^%d too large", logl);
  const int L = 1 << logl;
  BlockArgs a{};
  a.x = x;
  a.xs = xs;
  a.xlen = xlen;
  a.y = y;
  a.ys = ys;
  a.ylen = ylen;
  a.pre = overlap_save ? hlen - 1 : 0;
  a.step = L - a.pre;
  VS_REQUIRE(a.step > 0, "overlap-save: filter (%d) longer than the block (%d)", hlen, L);
  a.nblk = (ylen + a.step - 1) / a.step;
  a.h_per_signal = hs != 0;
  if (a.h_per_signal && (a.nblk & 1)) a.nblk++;  // never pair across filters
  a.nslots = static_cast<long long>(a.nblk) * batch;
  a.scale = 1.0f / static_cast<float>(L);
  DeviceBuffer spec;
  VS_TRY(filter_spectra(correlate, h, hlen, hs, a.h_per_signal ? batch : 1, logl,
                        spec, s));
  a.H = spec.as<float2>();
  vs_status st;
  const float2 *tw = fft::twiddles(logl, &st);
  if (!tw) return st;
  switch (logl) {
#define VS_CASE(LG) \
  case LG: launch_block_t<LG>(a, tw, s); break;
    VS_CASE(4) VS_CASE(5) VS_CASE(6) VS_CASE(7) VS_CASE(8) VS_CASE(9)
    VS_CASE(10) VS_CASE(11) VS_CASE(12) VS_CASE(13) VS_CASE(14)
#undef VS_CASE
    default:
      set_error("block convolution: unsupported block 2^%d", logl);
      return VS_ERR_UNSUPPORTED;
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// Real-block kernel or pair kernel for blocks of 2^logl samples.  Measured
// at x = 2^20, batch 64 (profiles/r2/conv_real_ab.md): the real-block kernel
// wins from L = 4096 on (1500 taps: 302 vs 288 Gsamples/s; 3000: 303 vs
// 228; 4096: 262 vs 242), the pair kernel at
// L = 2048 (1000 taps: 296 vs 284) where both stay L2-resident and the
// pair kernel skips the spectrum exchange.
bool use_real(int logl) {
  if (g_conv_real == 0 || logl < kRealMinLog) return false;
  return logl >= 12 || g_conv_real_all;
}

// Real-block path (real_conv_kernel): blocks of L = 2^logl real samples.
// `ylen` outputs per row land at y (row stride ys, `yroom` writable samples
// per row from y); accumulate adds them to what is there.
vs_status run_real(int correlate, bool overlap_save, const float *x, int xlen, int64_t xs,
                   const float *h, int hlen, int64_t hs, float *y, int64_t ys, int ylen,
                   int yroom, int accumulate, int batch, hipStream_t s,
                   const float4 *pq_pre = nullptr, int logl = 0) {
  if (logl) {
    // block fixed by a plan
  } else if (overlap_save) {
    logl = os_block_log(hlen);
  } else {
    logl = kRealMinLog;
    while ((1LL << logl) < ylen) logl++;
  }
  VS_REQUIRE(logl >= kRealMinLog && logl <= fft::kMaxLdsLog + 1,
             "real-block convolution: block 2^%d out of range", logl);
  const int L = 1 << logl;
  RealArgs a{};
  a.x = x;
  a.xs = xs;
  a.xlen = xlen;
  a.y = y;
  a.ys = ys;
  a.ylen = ylen;
  a.yroom = yroom;
  a.pq_per_signal = hs != 0;
  // history of at least h - 1 samples, rounded up to even: every block's
  // first valid output then starts a sample pair, which store_real's
  // descriptor-range stores need (a b64 store whose first dword lies before
  // the range is dropped whole -- measured: odd h - 1 lost each block's
  // first output)
  a.pre = overlap_save ? (hlen - 1 + 1) & ~1 : 0;
  a.step = L - a.pre;
  VS_REQUIRE(a.step > 0 && hlen <= L, "real-block convolution: filter (%d) longer than the block (%d)",
             hlen, L);
  a.nblk = (ylen + a.step - 1) / a.step;
  a.accumulate = accumulate;
  const long long nblocks = static_cast<long long>(a.nblk) * batch;
  VS_REQUIRE(batch <= kMaxGridY, "real-block convolution: batch %d > %lld per launch", batch,
             kMaxGridY);
  const int nfilt = hs ? batch : 1;
  switch (logl - 1) {
#define VS_CASE(LG, EP) \
  case LG: return run_real_t<LG, EP>(correlate, h, hlen, hs, nfilt, a, nblocks, pq_pre, s);
    VS_CASE(6, 0) VS_CASE(7, 0) VS_CASE(8, 0) VS_CASE(9, 0) VS_CASE(10, 0) VS_CASE(11, 0)
    VS_CASE(12, 0)
#undef VS_CASE
    case 13:
      return run_real_t<13, 32>(correlate, h, hlen, hs, nfilt, a, nblocks, pq_pre, s);
    case 14:
      return run_real_t<14, 0>(correlate, h, hlen, hs, nfilt, a, nblocks, pq_pre, s);
  }
  set_error("real-block convolution: unsupported block 2^%d", logl);
  return VS_ERR_UNSUPPORTED;
}

// Filters too long for one overlap-save block: uniformly partitioned
// overlap-save (fdl_*_kernel above).  Blocks of L = 2^fdl_block_log(hlen) samples, B =
// L / 2 taps per partition.  `pq_pre`: the partitions' P / Q tables when a
// plan holds them.  Signals go through in groups whose spectra (Z and Y:
// 16 bytes per sample and per output) fit kFdlScratch.
constexpr size_t kFdlScratch = static_cast<size_t>(6) << 30;

template <int LOGM, int EP>
vs_status run_fdl_t(int correlate, const float *x, int xlen, int64_t xs, const float *h,
                    int hlen, int64_t hs, float *y, int64_t ys, int ylen, int batch,
                    hipStream_t s, const float4 *pq_pre) {
  using PL = Plan<LOGM, EP>;
  constexpr int M = PL::N, B = M;
  const int parts = (hlen + B - 1) / B;
  const int nblk = (ylen + B - 1) / B;
  // source block b holds x[(b - 1) B, (b + 1) B): all zero from (xlen - 1) / B + 2 on
  const int nsrc = std::min((xlen - 1) / B + 2, nblk);
  const int nfilt = hs ? batch : 1;
  vs_status st;
  const float2 *tw = fft::twiddles(LOGM, &st);
  if (!tw) return st;
  DeviceBuffer pq;
  const float4 *PQ = pq_pre;
  if (!PQ) {
    VS_TRY(pq.alloc(sizeof(float4) * M * static_cast<size_t>(parts) * nfilt, s));
    VS_TRY(launch_real_filter<LOGM>(correlate, h, hlen, hs, nfilt, pq.as<float4>(), s, B));
    PQ = pq.as<float4>();
  }
  const size_t per_sig = (static_cast<size_t>(nsrc) + nblk) * M * sizeof(float2);
  const int group = static_cast<int>(
      std::max<size_t>(1, std::min<size_t>({static_cast<size_t>(batch), kFdlScratch / per_sig,
                                            static_cast<size_t>(kMaxGridY)})));
  DeviceBuffer zy;
  VS_TRY(zy.alloc(per_sig * group, s));
  float2 *Z = zy.as<float2>(), *Y = Z + static_cast<size_t>(group) * nsrc * M;
  const bool buf = g_conv_buf && xlen < (1 << 29) && ylen < (1 << 29);
  log(2, "vs_conv1d: partitioned overlap-save, L=%d, %d partitions, %d + %d blocks, groups of %d",
      2 * M, parts, nsrc, nblk, group);
  for (int b0 = 0; b0 < batch; b0 += group) {
    const int nb = std::min(group, batch - b0);
    RealArgs a{};
    a.x = x + static_cast<int64_t>(b0) * xs;
    a.xs = xs;
    a.xlen = xlen;
    a.y = y + static_cast<int64_t>(b0) * ys;
    a.ys = ys;
    a.ylen = ylen;
    a.yroom = ylen;
    a.pre = B;
    a.step = B;
    a.nblk = nblk;
    const dim3 gf(static_cast<unsigned>(nsrc), static_cast<unsigned>(nb));
    const dim3 gi(static_cast<unsigned>(nblk), static_cast<unsigned>(nb));
    if (buf)
      hipLaunchKernelGGL((fdl_forward_kernel<LOGM, EP, true>), gf, dim3(PL::TPS), 0, s, a, Z, tw);
    else
      hipLaunchKernelGGL((fdl_forward_kernel<LOGM, EP, false>), gf, dim3(PL::TPS), 0, s, a, Z, tw);
    FdlMac m{Z, PQ + (hs ? static_cast<size_t>(b0) * parts * M : 0), Y, nsrc, nblk, parts, M,
             hs != 0};
    if (g_fdl_mac_lds) {
      // chunks of 8 partitions while that is all of them, else 16 (47 KiB of LDS, three
      // workgroups per CU: 25 partitions run 67 Gsamples/s against 65 with chunks of 32
      // and 58 with chunks of 8, profiles/r3/conv/fdl.md)
      const int pc_max = g_fdl_mac_chunk ? g_fdl_mac_chunk
                                         : parts <= 8 ? 8 : 16;
      const size_t lds = static_cast<size_t>(kFdlLdsTile + pc_max - 1) * 2 * kFdlLdsBins * sizeof(float2);
      const dim3 gm((M / 2 + 1 + kFdlLdsBins - 1) / kFdlLdsBins,
                    static_cast<unsigned>((nblk + kFdlLdsTile - 1) / kFdlLdsTile),
                    static_cast<unsigned>(nb));
      if (pc_max == 8)
        hipLaunchKernelGGL(fdl_mac_lds_kernel<8>, gm, dim3(256), lds, s, m);
      else if (pc_max == 16)
        hipLaunchKernelGGL(fdl_mac_lds_kernel<16>, gm, dim3(256), lds, s, m);
      else
        hipLaunchKernelGGL(fdl_mac_lds_kernel<kFdlLdsChunk>, gm, dim3(256), lds, s, m);
    } else {
      hipLaunchKernelGGL(fdl_mac_kernel,
                         dim3((M / 2 + 1 + 255) / 256,
                              static_cast<unsigned>((nblk + kFdlTile - 1) / kFdlTile),
                              static_cast<unsigned>(nb)),
                         dim3(256), 0, s, m);
    }
    if (buf)
      hipLaunchKernelGGL((fdl_inverse_kernel<LOGM, EP, true>), gi, dim3(PL::TPS), 0, s, a, Y, tw);
    else
      hipLaunchKernelGGL((fdl_inverse_kernel<LOGM, EP, false>), gi, dim3(PL::TPS), 0, s, a, Y, tw);
    VS_HIP(hipGetLastError());
  }
  return VS_OK;
}

// log2 of the block of the partitioned path: vs_tune_set("fdl_block_log") 13 / 14 / 15, or
// 0 = by filter length: L = 16384 up to 20 partitions of 8192 taps, L = 32768 beyond (the
// larger transforms run slower per sample -- one workgroup per CU -- but halve the spectral
// accumulation: per-signal filters of 65,536 / 200,000 / 400,000 taps at 2^20 x 64 run
// 95 / 59 / 35 Gsamples/s on L = 16384 and 86 / 65 / 46 on L = 32768,
// profiles/r3/conv/fdl.md).
thread_local int g_fdl_log = 0;

int fdl_block_log(int hlen) {
  if (g_fdl_log) return g_fdl_log;
  return hlen > kFdlMaxParts * 8192 ? 15 : 14;
}
int fdl_part_taps(int hlen) { return 1 << (fdl_block_log(hlen) - 1); }

vs_status run_partitioned(int correlate, const float *x, int xlen, int64_t xs,
                          const float *h, int hlen, int64_t hs, float *y, int64_t ys, int ylen,
                          int batch, hipStream_t s, const float4 *pq_pre = nullptr,
                          int logl = 0) {
  const int l = logl ? logl : fdl_block_log(hlen);
  if (l == 13)
    return run_fdl_t<12, 0>(correlate, x, xlen, xs, h, hlen, hs, y, ys, ylen, batch, s, pq_pre);
  if (l == 15)
    return run_fdl_t<14, 0>(correlate, x, xlen, xs, h, hlen, hs, y, ys, ylen, batch, s, pq_pre);
  return run_fdl_t<13, 32>(correlate, x, xlen, xs, h, hlen, hs, y, ys, ylen, batch, s, pq_pre);
}

vs_status run_fft_large(int correlate, const float *x, int xlen, int64_t xs,
                        const float *h, int hlen, int64_t hs, float *y, int64_t ys,
                        int batch, hipStream_t s) {
  const int ylen = xlen + hlen - 1;
  int logm = 1;
  while ((1LL << logm) < ylen) logm++;
  VS_REQUIRE(logm <= fft::kMaxLog, "FFT convolution: padded length 2^%d too large",
             logm);
  int log1, log2;
  fft::four_step_split(logm, &log1, &log2);
  const long long M = 1LL << logm;
  const long long npairs = (batch + 1) / 2;
  const bool per = hs != 0;
  // One filter for all signals (per-signal filters take the partitioned
  // overlap-save path, vs_conv1d).
  VS_REQUIRE(!per, "FFT convolution: per-signal filters need the overlap-save path");
  DeviceBuffer hz, z;
  VS_TRY(hz.alloc(M * sizeof(float2), s));
  VS_TRY(z.alloc(M * npairs * sizeof(float2), s));
  hipLaunchKernelGGL(pad_filter_kernel, dim3(elementwise_grid(M, 256)), dim3(256), 0,
                     s, h, hlen, hs, correlate, logm, 1, hz.as<float2>());
  VS_TRY(fft::launch_cols(logm, false, hz.as<float2>(), hz.as<float2>(), 1, s));
  VS_TRY(fft::launch_c2c_lds(log2, false, hz.as<float2>(), hz.as<float2>(), 1 << log1, s));
  if (g_conv_fused4) {
    return fft::conv_four_step(logm, x, xlen, xs, batch, hz.as<float2>(), y, ys, ylen,
                               z.as<float2>(), s);
  }
  hipLaunchKernelGGL(pack_pairs_kernel, dim3(elementwise_grid(M * npairs, 256)),
                     dim3(256), 0, s, x, xlen, xs, batch, logm, npairs, z.as<float2>());
  VS_TRY(fft::launch_cols(logm, false, z.as<float2>(), z.as<float2>(), npairs, s));
  VS_TRY(fft::launch_c2c_lds(log2, false, z.as<float2>(), z.as<float2>(),
                             static_cast<int>(npairs << log1), s));
  hipLaunchKernelGGL(spectrum_mul_kernel, dim3(elementwise_grid(M * npairs, 256)),
                     dim3(256), 0, s, z.as<float2>(), hz.as<float2>(), logm, npairs, 0);
  VS_TRY(fft::launch_c2c_lds(log2, true, z.as<float2>(), z.as<float2>(),
                             static_cast<int>(npairs << log1), s));
  VS_TRY(fft::launch_cols(logm, true, z.as<float2>(), z.as<float2>(), npairs, s));
  hipLaunchKernelGGL(unpack_pairs_kernel, dim3(elementwise_grid(npairs * ylen, 256)),
                     dim3(256), 0, s, z.as<float2>(), logm, npairs, batch, y, ys, ylen,
                     1.0f / static_cast<float>(M));
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // namespace conv
}  // namespace vs

// vs_tune_set keys of the wavelet kernels (wavelet.hip)
namespace vs {
namespace wav {
bool tune(const char *key, int value);
void tune_reset();
}
}  // namespace vs

using namespace vs;

extern "C" {

#ifdef VS_CONV_STAMPS
#include "csrc/diag/conv_probes.inc"
#endif

int vs_conv1d_select(int64_t xlen, int hlen, int batch) {
  return conv::select(xlen, hlen, batch);
}

int vs_conv1d_os_block(int hlen) { return 1 << conv::os_block_log(hlen); }

}  // extern "C"

struct vs_conv_plan {
  int algo, correlate;
  int64_t xlen;
  int hlen, nfilt;
  bool overlap_save;  // real plans: overlap-save blocks vs one block
  int logl;           // real plans: block of 2^logl samples
  int parts;          // > 0: partitioned overlap-save, filter partitions
  float4 *pq;         // real plans: nfilt x max(parts, 1) x 2^(logl-1) P / Q entries
  float *h;           // other plans: nfilt x hlen taps
};

extern "C" {

vs_status vs_conv1d_plan_create(int algo, int correlate, int64_t xlen, const float *h, int hlen,
                                int64_t hs, int nfilt, vs_conv_plan **plan,
                                vs_stream_t stream) {
  VS_REQUIRE(plan && h, "vs_conv1d_plan_create: null pointer");
  *plan = nullptr;
  VS_REQUIRE(xlen > 0 && hlen > 0 && nfilt >= 1, "vs_conv1d_plan_create: empty shape");
  VS_REQUIRE(nfilt == 1 || hs >= hlen, "vs_conv1d_plan_create: filter stride < filter length");
  VS_REQUIRE(hlen < (1 << 30), "vs_conv1d_plan_create: filter of %d taps too long", hlen);
  const long long ylen = static_cast<long long>(xlen) + hlen - 1;
  auto s = static_cast<hipStream_t>(stream);
  if (algo == VS_CONV_AUTO) algo = conv::select(xlen, hlen, nfilt);
  // rows cut into pieces (vs_conv1d_plan_execute) run overlap-save blocks
  if (ylen > conv::max_call_out() && algo == VS_CONV_FFT) algo = VS_CONV_OVERLAP_SAVE;
  VS_REQUIRE(algo >= VS_CONV_DIRECT && algo <= VS_CONV_OVERLAP_SAVE,
             "vs_conv1d_plan_create: unknown algorithm %d", algo);
  // The real-block path vs_conv1d would take for this shape, if any
  int logl = 0, parts = 0;
  bool os = false;
  if (algo == VS_CONV_OVERLAP_SAVE) {
    const int l = conv::os_block_log(hlen);
    if (conv::os_single_block(hlen)) {
      if (conv::use_real(l)) logl = l, os = true;
    } else {  // partitioned: one P / Q table per partition
      logl = conv::fdl_block_log(hlen);
      parts = (hlen + (1 << (logl - 1)) - 1) >> (logl - 1);
      os = true;
    }
  } else if (algo == VS_CONV_FFT) {
    int lm = 1;
    while ((1LL << lm) < ylen) lm++;
    if (lm <= fft::kMaxLdsLog + 1 && conv::use_real(lm)) {
      logl = conv::kRealMinLog;
      while ((1LL << logl) < ylen) logl++;
    }
  }
  auto *p = new vs_conv_plan{algo, correlate, xlen, hlen, nfilt, os, logl, parts, nullptr, nullptr};
  vs_status st = VS_OK;
  if (logl) {
    const size_t n = (static_cast<size_t>(1) << (logl - 1)) * nfilt * std::max(parts, 1);
    const int part_taps = parts ? 1 << (logl - 1) : 0;
    if (hipMalloc(&p->pq, n * sizeof(float4)) != hipSuccess) {
      (void)hipGetLastError();
      st = VS_ERR_ALLOC;
      set_error("vs_conv1d_plan_create: out of device memory (%zu B)", n * sizeof(float4));
    } else {
      switch (logl - 1) {
#define VS_CASE(LG)                                                                           \
  case LG:                                                                                    \
    st = conv::launch_real_filter<LG>(correlate, h, hlen, nfilt > 1 ? hs : 0, nfilt, p->pq, s, \
                                      part_taps);                                              \
    break;
        VS_CASE(6) VS_CASE(7) VS_CASE(8) VS_CASE(9) VS_CASE(10) VS_CASE(11) VS_CASE(12)
        VS_CASE(13) VS_CASE(14)
#undef VS_CASE
        default:
          st = VS_ERR_UNSUPPORTED;
          set_error("vs_conv1d_plan_create: unsupported block 2^%d", logl);
      }
    }
  } else {
    const size_t n = static_cast<size_t>(hlen) * nfilt;
    if (hipMalloc(&p->h, n * sizeof(float)) != hipSuccess) {
      (void)hipGetLastError();
      st = VS_ERR_ALLOC;
      set_error("vs_conv1d_plan_create: out of device memory (%zu B)", n * sizeof(float));
    } else if (hipMemcpy2DAsync(p->h, hlen * sizeof(float), h,
                                (nfilt > 1 ? hs : hlen) * sizeof(float), hlen * sizeof(float),
                                nfilt, hipMemcpyDefault, s) != hipSuccess) {
      (void)hipGetLastError();
      st = VS_ERR_HIP;
      set_error("vs_conv1d_plan_create: filter copy failed");
    }
  }
  if (st != VS_OK) {
    vs_conv1d_plan_destroy(p);
    return st;
  }
  *plan = p;
  return VS_OK;
}

vs_status vs_conv1d_plan_execute(const vs_conv_plan *p, const float *x, int64_t xs, float *y,
                                 int64_t ys, int batch, vs_stream_t stream) {
  VS_REQUIRE(p && x && y, "vs_conv1d_plan_execute: null pointer");
  VS_REQUIRE(batch >= 0, "vs_conv1d_plan_execute: negative batch");
  VS_REQUIRE(p->nfilt == 1 || batch == p->nfilt,
             "vs_conv1d_plan_execute: plan has %d per-signal filters, batch %d", p->nfilt,
             batch);
  if (batch == 0) return VS_OK;
  const long long ylen = static_cast<long long>(p->xlen) + p->hlen - 1;
  VS_REQUIRE(batch <= 1 || (xs >= p->xlen && ys >= ylen),
             "vs_conv1d_plan_execute: row strides smaller than the rows");
  auto s = static_cast<hipStream_t>(stream);
  if (!p->pq)
    return vs_conv1d(p->algo, p->correlate, x, p->xlen, xs, p->h, p->hlen,
                     p->nfilt > 1 ? p->hlen : 0, y, ys, batch, stream);
  if (batch > kMaxGridY && !p->parts) {
    VS_REQUIRE(p->nfilt == 1, "vs_conv1d_plan_execute: per-signal batch > %lld", kMaxGridY);
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_conv1d_plan_execute(p, x + b0 * xs, xs, y + b0 * ys, ys, nb, stream);
    });
  }
  // h is not read when the spectra are precomputed; hs only flags per-signal P / Q.
  // One launch sequence over x[x0, x0 + xl) writing its first `outs` outputs at yy.
  const int64_t hs = p->nfilt > 1 ? p->hlen : 0;
  const auto run = [&](const float *xx, int xl, float *yy, int outs) {
    if (p->parts)
      return conv::run_partitioned(p->correlate, xx, xl, xs, nullptr, p->hlen, hs, yy, ys, outs,
                                   batch, s, p->pq, p->logl);
    return conv::run_real(p->correlate, p->overlap_save, xx, xl, xs, nullptr, p->hlen, hs, yy, ys,
                          outs, outs, 0, batch, s, p->pq, p->logl);
  };
  if (ylen <= conv::max_call_out())
    return run(x, static_cast<int>(p->xlen), y, static_cast<int>(ylen));
  // long rows: the pieces of vs_conv1d, last to first, with the plan's spectra
  const long long piece = conv::piece_out();
  for (long long c = (ylen + piece - 1) / piece - 1; c >= 0; c--) {
    const long long o0 = c * piece;
    const long long olen = std::min(piece, ylen - o0);
    const long long x0 = std::max<long long>(0, o0 - (p->hlen - 1));
    const long long x1 = std::min<long long>(p->xlen, o0 + olen);
    VS_TRY(run(x + x0, static_cast<int>(x1 - x0), y + x0, static_cast<int>(o0 - x0 + olen)));
  }
  return VS_OK;
}

vs_status vs_conv1d_plan_info(const vs_conv_plan *p, int *algo, int *precomputed) {
  VS_REQUIRE(p, "vs_conv1d_plan_info: null plan");
  if (algo) *algo = p->algo;
  if (precomputed) *precomputed = p->pq ? 1 : 0;
  return VS_OK;
}

void vs_conv1d_plan_destroy(vs_conv_plan *p) {
  if (!p) return;
  if (p->pq) (void)hipFree(p->pq);
  if (p->h) (void)hipFree(p->h);
  delete p;
}

vs_status vs_tune_set(const char *key, int value) {
  VS_REQUIRE(key, "vs_tune_set: null key");
  if (std::strcmp(key, "os_block_log_max") == 0) {
    VS_REQUIRE(value >= 4 && value <= fft::kMaxLdsLog + 1, "os_block_log_max out of range");
    conv::g_os_log_max = value;
    return VS_OK;
  }
  if (std::strcmp(key, "os_block_extra") == 0) {
    VS_REQUIRE(value == 0 || (value >= 2 && value <= 4), "os_block_extra must be 0 or 2..4");
    conv::g_os_extra = value;
    return VS_OK;
  }
  if (std::strcmp(key, "conv_buffer") == 0) {
    conv::g_conv_buf = value != 0;
    return VS_OK;
  }
  if (std::strcmp(key, "conv_real") == 0) {
    VS_REQUIRE(value == 0 || value == 1, "conv_real must be 0 or 1");
    conv::g_conv_real = value;
    return VS_OK;
  }
  if (std::strcmp(key, "conv_fused4") == 0) {
    conv::g_conv_fused4 = value < 0 ? 1 : value != 0;
    return VS_OK;
  }
  if (std::strcmp(key, "conv_real_all") == 0) {
    conv::g_conv_real_all = value != 0;
    return VS_OK;
  }
  if (std::strcmp(key, "conv_piece_log") == 0) {
    VS_REQUIRE(value >= 10 && value <= 28, "conv_piece_log must be 10..28");
    conv::g_piece_log = value;
    return VS_OK;
  }
  if (std::strcmp(key, "fdl_block_log") == 0) {
    VS_REQUIRE(value == 0 || (value >= 13 && value <= 15), "fdl_block_log must be 0 (by filter length), 13, 14 or 15");
    conv::g_fdl_log = value;
    return VS_OK;
  }
  if (std::strcmp(key, "fdl_mac_chunk") == 0) {
    VS_REQUIRE(value == 0 || value == 8 || value == 16 || value == 32,
               "fdl_mac_chunk must be 0, 8, 16 or 32");
    conv::g_fdl_mac_chunk = value;
    return VS_OK;
  }
  if (std::strcmp(key, "fdl_mac_lds") == 0) {
    conv::g_fdl_mac_lds = value != 0;
    return VS_OK;
  }
  if (wav::tune(key, value)) return VS_OK;
  set_error("vs_tune_set: unknown key '%s'", key);
  return VS_ERR_INVALID;
}

void vs_tune_reset(void) {
  conv::g_os_log_max = fft::kMaxLdsLog + 1;
  conv::g_os_extra = 0;
  conv::g_conv_fused4 = 1;
  conv::g_conv_buf = 1;
  conv::g_conv_real = 1;
  conv::g_conv_real_all = 0;
  conv::g_fdl_log = 0;
  conv::g_fdl_mac_lds = 1;
  conv::g_fdl_mac_chunk = 0;
  conv::g_piece_log = 28;
  wav::tune_reset();
}

}  // extern "C"

namespace vs {
namespace conv {

// One launch sequence: lengths within the kernels' 32-bit indexing, the
// first `ylen` (<= xlen + hlen - 1) outputs of every row written.
vs_status dispatch(int algo, int correlate, const float *x, int xlen, int64_t xs,
                   const float *h, int hlen, int64_t hs, float *y, int64_t ys, int ylen,
                   int batch, hipStream_t s) {
  const long long full = static_cast<long long>(xlen) + hlen - 1;
  log(2, "vs_conv1d: x=%d h=%d batch=%d algo=%d outputs=%d", xlen, hlen, batch, algo, ylen);
  int lm = 1;
  while ((1LL << lm) < full) lm++;
  switch (algo) {
    case VS_CONV_DIRECT:
      return run_direct(correlate, x, xlen, xs, h, hlen, hs, y, ys, ylen, batch, s);
    case VS_CONV_OVERLAP_SAVE:
      if (os_single_block(hlen)) {
        if (use_real(os_block_log(hlen)))
          return run_real(correlate, true, x, xlen, xs, h, hlen, hs, y, ys, ylen, ylen, 0, batch,
                          s);
        return run_block(correlate, true, x, xlen, xs, h, hlen, hs, y, ys, ylen, batch, s);
      }
      log(1, "vs_conv1d: filter %d longer than an overlap-save block: %d partitions", hlen,
          (hlen + fdl_part_taps(hlen) - 1) / fdl_part_taps(hlen));
      return run_partitioned(correlate, x, xlen, xs, h, hlen, hs, y, ys, ylen, batch, s);
    case VS_CONV_FFT:
      if (lm <= fft::kMaxLdsLog || (lm == fft::kMaxLdsLog + 1 && use_real(lm))) {
        if (use_real(lm))
          return run_real(correlate, false, x, xlen, xs, h, hlen, hs, y, ys, ylen, ylen, 0, batch,
                          s);
        return run_block(correlate, false, x, xlen, xs, h, hlen, hs, y, ys, ylen, batch, s);
      }
      if (lm <= fft::kMaxLog && hs == 0 && ylen == full)
        return run_fft_large(correlate, x, xlen, xs, h, hlen, hs, y, ys, batch, s);
      // beyond the largest transform, one filter per signal, or a piece of a
      // longer row: overlap-save (partitioned when the filter needs it)
      log(1, "vs_conv1d: FFT of 2^%d%s: overlap-save", lm, hs ? " with per-signal filters" : "");
      return dispatch(VS_CONV_OVERLAP_SAVE, correlate, x, xlen, xs, h, hlen, hs, y, ys, ylen,
                      batch, s);
  }
  set_error("vs_conv1d: unknown algorithm %d", algo);
  return VS_ERR_INVALID;
}

}  // namespace conv
}  // namespace vs

extern "C" {

vs_status vs_conv1d(int algo, int correlate, const float *x, int64_t xlen,
                    int64_t xs, const float *h, int hlen, int64_t hs, float *y,
                    int64_t ys, int batch, vs_stream_t stream) {
  VS_REQUIRE(x && h && y, "vs_conv1d: null pointer");
  VS_REQUIRE(xlen > 0 && hlen > 0 && batch >= 0, "vs_conv1d: empty input");
  VS_REQUIRE(hlen < (1 << 30), "vs_conv1d: filter of %d taps too long", hlen);
  const long long ylen = static_cast<long long>(xlen) + hlen - 1;
  VS_REQUIRE(batch <= 1 || (xs >= xlen && ys >= ylen),
             "vs_conv1d: row strides smaller than the rows");
  VS_REQUIRE(hs == 0 || hs >= hlen, "vs_conv1d: filter stride < filter length");
  if (batch == 0) return VS_OK;
  auto s = static_cast<hipStream_t>(stream);
  if (algo == VS_CONV_AUTO) algo = conv::select(xlen, hlen, batch);
  VS_REQUIRE(algo >= VS_CONV_DIRECT && algo <= VS_CONV_OVERLAP_SAVE,
             "vs_conv1d: unknown algorithm %d", algo);
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_conv1d(algo, correlate, x + b0 * xs, xlen, xs, h + b0 * hs, hlen, hs,
                       y + b0 * ys, ys, nb, stream);
    });
  if (ylen <= conv::max_call_out())
    return conv::dispatch(algo, correlate, x, static_cast<int>(xlen), xs, h, hlen, hs, y, ys,
                          static_cast<int>(ylen), batch, s);
  // Long rows: pieces of 2^28 outputs, each the convolution of its x
  // samples and the hlen - 1 before them.  A piece writes from the first
  // output its x range produces -- the `skip` outputs before its own range
  // lack their history -- and stops at the end of its range; the pieces run
  // last to first, so the piece that owns those `skip` outputs overwrites
  // them afterwards (same stream).
  if (algo == VS_CONV_FFT) algo = VS_CONV_OVERLAP_SAVE;
  const long long piece = conv::piece_out();
  const long long pieces = (ylen + piece - 1) / piece;
  log(1, "vs_conv1d: x=%lld in %lld pieces of %lld outputs", static_cast<long long>(xlen), pieces,
      piece);
  for (long long c = pieces - 1; c >= 0; c--) {
    const long long o0 = c * piece;
    const long long olen = std::min(piece, ylen - o0);
    const long long x0 = std::max<long long>(0, o0 - (hlen - 1));
    const long long x1 = std::min<long long>(xlen, o0 + olen);
    const long long skip = o0 - x0;
    VS_TRY(conv::dispatch(algo, correlate, x + x0, static_cast<int>(x1 - x0), xs, h, hlen, hs,
                          y + x0, ys, static_cast<int>(skip + olen), batch, s));
  }
  return VS_OK;
}

}  // extern "C"
