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

#include <cstdint>
#include <cstring>

#include "csrc/kernels/device.h"
#include "csrc/kernels/fft_core.h"
#include "csrc/kernels/fft_plan.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace conv {
extern int g_conv_buf, g_conv_split;  // tuning knobs, defined below
namespace {

using fft::cmul;
using fft::Plan;
using fft::reg_index;

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
    if (n0 + i < ylen) yrow[n0 + i] = buf[i];
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
template <int HM>
__global__ __launch_bounds__(kDirThreads) void direct_small_kernel(
    const float *__restrict__ x, int xlen, int64_t xs, const float *__restrict__ h,
    int hlen, int64_t hs, float *__restrict__ y, int64_t ys, int ylen, int reverse) {
  constexpr int W = kDirOut + HM + 8;  // window floats (+ slack for the b128 reads)
  __shared__ __attribute__((aligned(16))) float sx[W];
  const int sig = blockIdx.y;
  const float *xrow = x + sig * xs;
  const float *hrow = h + sig * hs;
  const int n0 = blockIdx.x * kDirOut;
  // window: sx[i] = x[n0 - (HM - 1) + i]
  const int xbase = n0 - (HM - 1);
  for (int i = threadIdx.x; i < W; i += kDirThreads) {
    const int p = xbase + i;
    sx[i] = (p >= 0 && p < xlen) ? xrow[p] : 0.f;
  }
  float tap[HM];
#pragma unroll
  for (int m = 0; m < HM; m++)
    tap[m] = m < hlen ? (reverse ? hrow[hlen - 1 - m] : hrow[m]) : 0.f;
  __syncthreads();
  const int q0 = threadIdx.x * kDirPerThread;
  constexpr int NW = (kDirPerThread + HM - 1 + 3) / 4;  // float4 reads per lane
  float w[4 * NW];
#pragma unroll
  for (int c = 0; c < NW; c++) {
    const float4 v = *reinterpret_cast<const float4 *>(sx + q0 + 4 * c);
    w[4 * c] = v.x;
    w[4 * c + 1] = v.y;
    w[4 * c + 2] = v.z;
    w[4 * c + 3] = v.w;
  }
  // y[n0 + q0 + r] = sum_m tap[m] x[n0 + q0 + r - m] = sum_m tap[m] w[r - m + HM - 1]
  float acc[kDirPerThread];
#pragma unroll
  for (int r = 0; r < kDirPerThread; r++) {
    float a = 0.f;
#pragma unroll
    for (int m = 0; m < HM; m++) a = fmaf(tap[m], w[r - m + HM - 1], a);
    acc[r] = a;
  }
  store_outputs(acc, sx, y + sig * ys, n0, q0, ylen);
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
                                              4 * (base0 + a.pre + n), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(r.y * a.scale), w1,
                                              4 * (base1 + a.pre + n), 0, 0);
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
        if (q.ok0 && o0 < a.ylen) y0[o0] = r.x * a.scale;
        if (q.ok1 && o1 < a.ylen) y1[o1] = r.y * a.scale;
      }
  }
}

// One workgroup per block pair.  No barrier between the transforms: the
// forward transform's last LDS read is followed by a barrier inside it.
// SPLIT (16384 points): the LDS exchanges move real and imaginary parts one
// after the other through a 68 KiB float image instead of a 137 KiB float2
// one, so two workgroups share a CU (16 waves instead of 8, 128 VGPRs each)
// and one's HBM loads / stores and barriers overlap the other's butterflies.
template <int LOGN, bool BUF, bool SPLIT>
__global__ __launch_bounds__(Plan<LOGN>::TPS, SPLIT ? 4 : 1) void block_conv_kernel(
    BlockArgs a, const float2 *__restrict__ tw) {
  using PL = Plan<LOGN>;
  __shared__ std::conditional_t<SPLIT, float, float2> lds[PL::kLds];
  const int t = threadIdx.x;
  const PairPos q = pair_pos(a, blockIdx.x);
  float2 v[PL::E];
  load_pair<PL, BUF>(a, q, t, v);
  // every input load in flight before the first butterfly consumes one (the
  // scheduler otherwise splits them into dependent batches)
  __builtin_amdgcn_sched_barrier(0);
  fft::transform<PL, false, false>(v, lds, t, tw);
  // SPLIT has half the registers: keep the spectrum loads from being
  // hoisted into the forward transform (64 more live VGPRs)
  if constexpr (SPLIT) __builtin_amdgcn_sched_barrier(0);
  mul_spectrum<PL>(a, q, t, v);
  if constexpr (SPLIT) __builtin_amdgcn_sched_barrier(0);
  fft::transform<PL, true, true>(v, lds, t, tw);
  store_pair<PL, BUF>(a, q, t, v);
}

// Buffer addressing needs every byte offset of a row in 31 bits.
inline bool buffer_ok(const BlockArgs &a) {
  return g_conv_buf && a.xlen < (1 << 29) && a.ylen < (1 << 29);
}

template <int LOGN, bool SPLIT>
void launch_block_split(const BlockArgs &a, const float2 *tw, hipStream_t s) {
  const unsigned grid = static_cast<unsigned>((a.nslots + 1) / 2);
  if (buffer_ok(a))
    hipLaunchKernelGGL((block_conv_kernel<LOGN, true, SPLIT>), dim3(grid),
                       dim3(Plan<LOGN>::TPS), 0, s, a, tw);
  else
    hipLaunchKernelGGL((block_conv_kernel<LOGN, false, SPLIT>), dim3(grid),
                       dim3(Plan<LOGN>::TPS), 0, s, a, tw);
}

template <int LOGN>
void launch_block_t(const BlockArgs &a, const float2 *tw, hipStream_t s) {
  if constexpr (LOGN == fft::kMaxLdsLog) {
    if (g_conv_split) return launch_block_split<LOGN, true>(a, tw, s);
  }
  launch_block_split<LOGN, false>(a, tw, s);
}


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

// Tuning knob (vs_tune_set("os_block_log_max", n)): cap of the overlap-save
// block size, for A/B measurements.
int g_os_log_max = fft::kMaxLdsLog;
// Tuning knob (vs_tune_set("conv_buffer", 0/1)): buffer-descriptor loads and
// stores in the fused block kernels.
int g_conv_buf = 1;
// Tuning knob (vs_tune_set("conv_split", 0/1)): 16384-point block kernel with
// the split (real, then imaginary) LDS exchange, two workgroups per CU.
int g_conv_split = 0;

int os_block_log(int hlen) {
  // Reference block size 2^(floor(log2 M) + 2) (src/convolve.c:116-121),
  // raised to >= 2048 so every block amortises its transform over >= ~75%
  // useful outputs, capped at the single-workgroup LDS transform.
  int lg = 2;
  int m = hlen;
  while (m >>= 1) lg++;
  if (lg < 11) lg = 11;
  if (lg > g_os_log_max) lg = g_os_log_max;
  while ((1 << lg) <= hlen && lg < fft::kMaxLdsLog) lg++;  // must exceed h - 1
  return lg;
}

int select(int xlen, int hlen, int batch) {
  const long long ylen = static_cast<long long>(xlen) + hlen - 1;
  (void)batch;
  // Direct only for very short filters or signals: at x = 2^20 the fused
  // overlap-save kernel already beats the direct one from h = 16 on
  // (405 vs 267 Gsamples/s, profiles/r1/conv_sweep_v2.log).
  if (ylen <= 64 || hlen <= 8 || (hlen <= 32 && xlen < 4096)) return VS_CONV_DIRECT;
  const int los = os_block_log(hlen);
  const bool os_ok = (1 << los) - (hlen - 1) >= (1 << los) / 2;  // >= 50% useful
  int lm = 1;
  while ((1LL << lm) < ylen) lm++;
  if (lm <= fft::kMaxLdsLog && (!os_ok || ylen <= (1LL << los)))
    return VS_CONV_FFT;  // one block covers the whole output
  if (os_ok) return VS_CONV_OVERLAP_SAVE;
  return VS_CONV_FFT;
}

vs_status run_direct(int correlate, const float *x, int xlen, int64_t xs,
                     const float *h, int hlen, int64_t hs, float *y, int64_t ys,
                     int batch, hipStream_t s) {
  const int ylen = xlen + hlen - 1;
  const dim3 grid(static_cast<unsigned>((ylen + kDirOut - 1) / kDirOut),
                  static_cast<unsigned>(batch));
  if (hlen <= 8)
    hipLaunchKernelGGL(direct_small_kernel<8>, grid, dim3(kDirThreads), 0, s, x, xlen, xs, h,
                       hlen, hs, y, ys, ylen, correlate);
  else if (hlen <= 16)
    hipLaunchKernelGGL(direct_small_kernel<16>, grid, dim3(kDirThreads), 0, s, x, xlen, xs, h,
                       hlen, hs, y, ys, ylen, correlate);
  else if (hlen <= 32)
    hipLaunchKernelGGL(direct_small_kernel<32>, grid, dim3(kDirThreads), 0, s, x, xlen, xs, h,
                       hlen, hs, y, ys, ylen, correlate);
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
                    int64_t ys, int batch, hipStream_t s) {
  const int ylen = xlen + hlen - 1;
  int logl;
  if (overlap_save) {
    logl = os_block_log(hlen);
  } else {
    logl = 4;  // smallest instantiated transform
    while ((1 << logl) < ylen) logl++;
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
  // Filters: a complex signal per pair of outputs when filters differ; the
  // two members of a pair use different filters then, so fall back to one
  // signal per transform (imaginary part zero) in that case.
  if (per) {
    for (int b = 0; b < batch; b++) {
      VS_TRY(run_fft_large(correlate, x + b * xs, xlen, 0, h + b * hs, hlen, 0,
                           y + b * ys, ylen, 1, s));
    }
    return VS_OK;
  }
  DeviceBuffer hz, z;
  VS_TRY(hz.alloc(M * sizeof(float2), s));
  VS_TRY(z.alloc(M * npairs * sizeof(float2), s));
  hipLaunchKernelGGL(pad_filter_kernel, dim3(elementwise_grid(M, 256)), dim3(256), 0,
                     s, h, hlen, hs, correlate, logm, 1, hz.as<float2>());
  VS_TRY(fft::launch_cols(logm, false, hz.as<float2>(), hz.as<float2>(), 1, s));
  VS_TRY(fft::launch_c2c_lds(log2, false, hz.as<float2>(), hz.as<float2>(), 1 << log1, s));
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

using namespace vs;

extern "C" {

int vs_conv1d_select(int xlen, int hlen, int batch) {
  return conv::select(xlen, hlen, batch);
}

int vs_conv1d_os_block(int hlen) { return 1 << conv::os_block_log(hlen); }

vs_status vs_tune_set(const char *key, int value) {
  VS_REQUIRE(key, "vs_tune_set: null key");
  if (std::strcmp(key, "os_block_log_max") == 0) {
    VS_REQUIRE(value >= 4 && value <= fft::kMaxLdsLog, "os_block_log_max out of range");
    conv::g_os_log_max = value;
    return VS_OK;
  }
  if (std::strcmp(key, "conv_buffer") == 0) {
    conv::g_conv_buf = value != 0;
    return VS_OK;
  }
  if (std::strcmp(key, "conv_split") == 0) {
    conv::g_conv_split = value != 0;
    return VS_OK;
  }
  set_error("vs_tune_set: unknown key '%s'", key);
  return VS_ERR_INVALID;
}

vs_status vs_conv1d(int algo, int correlate, const float *x, int xlen,
                    int64_t xs, const float *h, int hlen, int64_t hs, float *y,
                    int64_t ys, int batch, vs_stream_t stream) {
  VS_REQUIRE(x && h && y, "vs_conv1d: null pointer");
  VS_REQUIRE(xlen > 0 && hlen > 0 && batch >= 0, "vs_conv1d: empty input");
  const long long ylen = static_cast<long long>(xlen) + hlen - 1;
  VS_REQUIRE(ylen < (1LL << 31), "vs_conv1d: output too long");
  VS_REQUIRE(batch <= 1 || (xs >= xlen && ys >= ylen),
             "vs_conv1d: row strides smaller than the rows");
  VS_REQUIRE(hs == 0 || hs >= hlen, "vs_conv1d: filter stride < filter length");
  if (batch == 0) return VS_OK;
  auto s = static_cast<hipStream_t>(stream);
  if (algo == VS_CONV_AUTO) algo = conv::select(xlen, hlen, batch);
  if (batch > kMaxGridY && algo != VS_CONV_OVERLAP_SAVE)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_conv1d(algo, correlate, x + b0 * xs, xlen, xs, h + b0 * hs, hlen, hs,
                       y + b0 * ys, ys, nb, stream);
    });
  log(2, "vs_conv1d: x=%d h=%d batch=%d algo=%d", xlen, hlen, batch, algo);
  switch (algo) {
    case VS_CONV_DIRECT:
      return conv::run_direct(correlate, x, xlen, xs, h, hlen, hs, y, ys, batch, s);
    case VS_CONV_OVERLAP_SAVE:
      if ((1 << conv::os_block_log(hlen)) > hlen - 1 + 16)
        return conv::run_block(correlate, true, x, xlen, xs, h, hlen, hs, y, ys,
                               batch, s);
      log(1, "vs_conv1d: filter %d too long for an overlap-save block, using FFT",
          hlen);
      [[fallthrough]];
    case VS_CONV_FFT: {
      int lm = 1;
      while ((1LL << lm) < ylen) lm++;
      if (lm <= fft::kMaxLdsLog)
        return conv::run_block(correlate, false, x, xlen, xs, h, hlen, hs, y, ys,
                               batch, s);
      return conv::run_fft_large(correlate, x, xlen, xs, h, hlen, hs, y, ys, batch, s);
    }
  }
  set_error("vs_conv1d: unknown algorithm %d", algo);
  return VS_ERR_INVALID;
}

}  // extern "C"
