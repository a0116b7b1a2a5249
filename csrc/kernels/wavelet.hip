// Decimated and stationary (a trous) wavelet transforms
// over the Daubechies / Symlet / Coiflet banks.
//
//   * single level (vs_dwt / vs_swt): a 256-thread block owns a tile of 1024
//     outputs of one signal, stages the input window (tile + filter support,
//     boundary extension applied on load) in LDS and every lane produces 4
//     outputs.  The SWT touches only the `order` non-zero taps of the dilated
//     filter (the reference expands it to order * 2^(level-1) taps,
//     src/wavelet.c:211-246).  Taps live in the kernel-argument segment and
//     are read with scalar loads.
//   * multi-level (vs_swt_multilevel / vs_dwt_multilevel): one workgroup per
//     signal keeps the running low-pass band in LDS across all levels and only
//     writes each level's high band (and the final low band) to HBM: one HBM
//     read of the input for L levels instead of L.
//
// Extension past the end of the signal follows the reference
// (src/wavelet.c:248-269): periodic src[t % len], mirror
// src[len - 1 - t % len], constant src[len - 1], zero.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "csrc/data/wavelet_tables.h"
#include "csrc/kernels/device.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace wav {
namespace {

constexpr int kMaxOrder = wavelet_tables::kMaxOrder;

struct Taps {
  float lp[kMaxOrder];
  float hp[kMaxOrder];
  int order;
};

template <class I>
__device__ __forceinline__ I ext_index(I idx, I len, int ext) {
  // Returns the source index for position idx (idx >= 0), or -1 for zero.
  if (idx < len) return idx;
  const I t = idx - len;
  switch (ext) {
    case EXTENSION_TYPE_PERIODIC: return t % len;
    case EXTENSION_TYPE_MIRROR: return len - 1 - (t % len);
    case EXTENSION_TYPE_CONSTANT: return len - 1;
    default: return -1;
  }
}

template <class P, class I>
__device__ __forceinline__ float ext_load(const P *src, I idx, I len, int ext) {
  const I j = ext_index(idx, len, ext);
  return j < 0 ? 0.f : static_cast<float>(src[j]);
}

// Workgroup barrier that orders LDS only: __syncthreads() also waits for the
// wave's outstanding global stores (vmcnt), i.e. for the high band of the
// level just written, at every level.  The levels only exchange data
// through LDS.  (Measured on 65536 x 1024, db8 x 8 levels: 0.503 vs 0.509 ms,
// within noise -- the stores are not what a level waits for.)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

constexpr int kThreads = 256;
constexpr int kPer = 4;
constexpr int kTile = kThreads * kPer;  // outputs per block

// One decimated level: hi/lo[k] = sum_j hp/lp[j] * x~[2k + j], k < len/2.
__global__ __launch_bounds__(kThreads) void dwt_kernel(
    Taps taps, int ext, const float *__restrict__ src, int64_t len, int64_t ss,
    float *__restrict__ hi, float *__restrict__ lo, int64_t os) {
  __shared__ float s[2 * kTile + kMaxOrder];
  const float *x = src + blockIdx.y * ss;
  const int64_t half = len / 2;
  const int64_t k0 = static_cast<int64_t>(blockIdx.x) * kTile;
  const int span = 2 * kTile + taps.order;
  for (int i = threadIdx.x; i < span; i += kThreads) {
    const int64_t idx = 2 * k0 + i;
    s[i] = idx < len + taps.order ? ext_load(x, idx, len, ext) : 0.f;
  }
  __syncthreads();
  float* h = hi + blockIdx.y * os;
  float* l = lo + blockIdx.y * os;
#pragma unroll
  for (int q = 0; q < kPer; q++) {
    const int kk = threadIdx.x + q * kThreads;
    float sh = 0.f, sl = 0.f;
    for (int j = 0; j < taps.order; j++) {
      const float v = s[2 * kk + j];
      sh = fmaf(taps.hp[j], v, sh);
      sl = fmaf(taps.lp[j], v, sl);
    }
    if (k0 + kk < half) {
      h[k0 + kk] = sh;
      l[k0 + kk] = sl;
    }
  }
}

// One stationary level with dilation `dil`: out[i] = sum_r c[r] x~[i + r dil].
// The LDS window is kTile + (order-1)*dil samples; launched only when it fits.
constexpr int kSwtLds = 12288;

__global__ __launch_bounds__(kThreads) void swt_kernel(
    Taps taps, int ext, int dil, const float *__restrict__ src, int64_t len,
    int64_t ss, float *__restrict__ hi, int64_t hs, float *__restrict__ lo,
    int64_t ls) {
  __shared__ float s[kSwtLds];
  const float *x = src + blockIdx.y * ss;
  const int64_t i0 = static_cast<int64_t>(blockIdx.x) * kTile;
  const int span = kTile + (taps.order - 1) * dil;
  for (int i = threadIdx.x; i < span; i += kThreads)
    s[i] = ext_load(x, i0 + i, len, ext);
  __syncthreads();
  float* h = hi + blockIdx.y * hs;
  float* l = lo + blockIdx.y * ls;
#pragma unroll
  for (int q = 0; q < kPer; q++) {
    const int ii = threadIdx.x + q * kThreads;
    float sh = 0.f, sl = 0.f;
    for (int r = 0; r < taps.order; r++) {
      const float v = s[ii + r * dil];
      sh = fmaf(taps.hp[r], v, sh);
      sl = fmaf(taps.lp[r], v, sl);
    }
    if (i0 + ii < len) {
      h[i0 + ii] = sh;
      l[i0 + ii] = sl;
    }
  }
}

// Same without LDS staging, for dilations whose window does not fit.
__global__ __launch_bounds__(kThreads) void swt_global_kernel(
    Taps taps, int ext, int dil, const float *__restrict__ src, int64_t len,
    int64_t ss, float *__restrict__ hi, int64_t hs, float *__restrict__ lo,
    int64_t ls) {
  const float *x = src + blockIdx.y * ss;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  if (i >= len) return;
  float sh = 0.f, sl = 0.f;
  for (int r = 0; r < taps.order; r++) {
    const float v = ext_load(x, i + static_cast<int64_t>(r) * dil, len, ext);
    sh = fmaf(taps.hp[r], v, sh);
    sl = fmaf(taps.lp[r], v, sl);
  }
  hi[blockIdx.y * hs + i] = sh;
  lo[blockIdx.y * ls + i] = sl;
}

// All `levels` stationary levels of one signal in LDS.  Each level first
// materialises the boundary extension of the current band behind it (so the
// tap loop is plain LDS reads with no index arithmetic), then every lane
// produces outputs i = tid + k * blockDim: the high band goes straight to
// HBM (coalesced), the low band to the other LDS buffer.
constexpr int kMultiMax = 8192;   // samples per signal held in LDS
constexpr int kMultiExt = 4096;   // room for the extension (order-1) 2^(L-1)

__global__ __launch_bounds__(256) void swt_multi_kernel(
    Taps taps, int ext, int levels, const float *__restrict__ src, int len,
    float *__restrict__ hi, int64_t hs, float *__restrict__ lo, int64_t ls) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int stride = len + ((taps.order - 1) << (levels - 1));
  float *band0 = smem, *band1 = smem + stride;
  const int64_t sig = blockIdx.x;
  const float *x = src + sig * len;
  for (int i = threadIdx.x; i < len; i += blockDim.x) band0[i] = x[i];
  float *in = band0, *out = band1;
  for (int l = 0; l < levels; l++) {
    const int dil = 1 << l;
    const int halo = (taps.order - 1) * dil;
    __syncthreads();  // band complete
    for (int t = threadIdx.x; t < halo; t += blockDim.x) {
      const int j = ext_index(len + t, len, ext);
      in[len + t] = j < 0 ? 0.f : in[j];
    }
    __syncthreads();
    float *hrow = hi + sig * hs + static_cast<int64_t>(l) * len;
    for (int i = threadIdx.x; i < len; i += blockDim.x) {
      float sh = 0.f, sl = 0.f;
      for (int r = 0; r < taps.order; r++) {
        const float v = in[i + r * dil];
        sh = fmaf(taps.hp[r], v, sh);
        sl = fmaf(taps.lp[r], v, sl);
      }
      hrow[i] = sh;
      out[i] = sl;
    }
    float *t = in;
    in = out;
    out = t;
  }
  __syncthreads();
  float *lrow = lo + sig * ls;
  for (int i = threadIdx.x; i < len; i += blockDim.x) lrow[i] = in[i];
}

// All levels of one signal in LDS with compile-time filter length and four
// consecutive outputs per lane (len % 4 == 0): taps in registers, 16-byte LDS
// reads of the input window (one window for dilation 1 and 2, one float4 per
// tap from dilation 4 on), 16-byte stores.  The boundary extension of the
// next level's input is written by the lanes that produce it, in the same
// pass:
//   periodic: in[len + t] = in[t]          -> the float4 at i0 < halo is also
//                                              stored at len + i0;
//   mirror:   in[len + t] = in[len - 1 - t] -> the float4 at i0 is stored
//                                              reversed at 2 len - 4 - i0;
//   zero:     the halo regions are zeroed once;
//   constant: one broadcast fill phase per level (the only extra barrier).
// No modulo / per-element extension code runs, each level costs one barrier,
// and the last level writes the low band straight to HBM.  Needs
// len % 4 == 0.
// PMC (db16, 16384 x 1024): a kernel with a separate modulo halo fill per
// level issued ~4x the VALU instructions of its FMAs, most of them in that
// fill (profiles/r2/swt/README.md).
template <int ORDER, bool NT, int SIGS>
__global__ __launch_bounds__(256) void swt_fused_kernel(
    Taps taps, int ext, int levels, const float *__restrict__ src, int len,
    float *__restrict__ hi, int64_t hs, float *__restrict__ lo, int64_t ls, int batch) {
  // SIGS signals per workgroup, interleaved lane by lane: every lane carries
  // SIGS independent float4 chains through each level and the level barrier
  // is shared.
  extern __shared__ __attribute__((aligned(16))) float smemf[];
  const int stride = (len + ((ORDER - 1) << (levels - 1)) + 2 * ORDER + 8 + 3) & ~3;
  // a last workgroup short of signals repeats the last one (same values
  // written twice) so the SIGS chains stay branch-free
  const int64_t sig0 = static_cast<int64_t>(blockIdx.x) * SIGS;
  const int64_t sig_last = batch - 1;
  const int len4 = len >> 2;
  float hp[ORDER], lp[ORDER];
#pragma unroll
  for (int r = 0; r < ORDER; r++) {
    hp[r] = taps.hp[r];
    lp[r] = taps.lp[r];
  }
  if (ext == EXTENSION_TYPE_ZERO) {
    const int z4 = (stride - len) >> 2;
    for (int b = 0; b < 2 * SIGS; b++)
      for (int i = threadIdx.x; i < z4; i += blockDim.x)
        reinterpret_cast<float4 *>(smemf + b * stride + len)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // Stores the float4 `v` at output position i0 of band `b` plus its image in
  // the extension region for a consumer needing `halo` extension samples.
  // The extension repeats with period len (reference src/wavelet.c:248-269:
  // periodic src[t % len], mirror src[len - 1 - t % len]), so a halo longer
  // than the signal takes one image per period.
  const auto put = [&](float *b, int i0, float4 v, int halo) {
    reinterpret_cast<float4 *>(b)[i0 >> 2] = v;
    if (ext == EXTENSION_TYPE_PERIODIC) {
      for (int t = i0; t < halo; t += len) reinterpret_cast<float4 *>(b + len + t)[0] = v;
    } else if (ext == EXTENSION_TYPE_MIRROR) {
      const float4 r = make_float4(v.w, v.z, v.y, v.x);
      for (int t = len - 4 - i0; t < halo; t += len)
        reinterpret_cast<float4 *>(b + len + t)[0] = r;
    }
  };
  // bands of signal g: smemf + (2 g + parity) stride
#pragma unroll
  for (int g = 0; g < SIGS; g++) {
    const float4 *x4 =
        reinterpret_cast<const float4 *>(src + min(sig0 + g, sig_last) * len);
    for (int q = threadIdx.x; q < len4; q += blockDim.x) {
      float4 v;
      if (NT) {  // read once: keep it out of the caches the stores stream through
        typedef float native4 __attribute__((ext_vector_type(4)));
        const native4 nv = __builtin_nontemporal_load(reinterpret_cast<const native4 *>(x4) + q);
        v = make_float4(nv.x, nv.y, nv.z, nv.w);
      } else {
        v = x4[q];
      }
      put(smemf + 2 * g * stride, 4 * q, v, ORDER - 1);
    }
  }
  int par = 0;
  for (int l = 0; l < levels; l++) {
    const int dil = 1 << l;
    lds_barrier();  // input bands and their extensions complete
    if (ext == EXTENSION_TYPE_CONSTANT) {
      for (int g = 0; g < SIGS; g++) {
        float *in = smemf + (2 * g + par) * stride;
        const float c = in[len - 1];
        for (int t = threadIdx.x; t < (ORDER - 1) * dil; t += blockDim.x) in[len + t] = c;
      }
      lds_barrier();
    }
    const bool last = l == levels - 1;
    const int next_halo = (ORDER - 1) * dil * 2;
    for (int q = threadIdx.x; q < len4; q += blockDim.x) {
      const int i0 = 4 * q;
#pragma unroll
      for (int g = 0; g < SIGS; g++) {
        const float *in = smemf + (2 * g + par) * stride;
        float *out = smemf + (2 * g + (par ^ 1)) * stride;
        const int64_t sig = min(sig0 + g, sig_last);
        float sh[4] = {0.f, 0.f, 0.f, 0.f}, sl[4] = {0.f, 0.f, 0.f, 0.f};
        if (dil <= 2) {
          constexpr int W = (4 + 2 * (ORDER - 1) + 3) / 4;
          float w[4 * W];
#pragma unroll
          for (int c = 0; c < W; c++) {
            const float4 v = reinterpret_cast<const float4 *>(in + i0)[c];
            w[4 * c] = v.x;
            w[4 * c + 1] = v.y;
            w[4 * c + 2] = v.z;
            w[4 * c + 3] = v.w;
          }
          if (dil == 1) {
#pragma unroll
            for (int r = 0; r < ORDER; r++)
#pragma unroll
              for (int e = 0; e < 4; e++) {
                sh[e] = fmaf(hp[r], w[r + e], sh[e]);
                sl[e] = fmaf(lp[r], w[r + e], sl[e]);
              }
          } else {
#pragma unroll
            for (int r = 0; r < ORDER; r++)
#pragma unroll
              for (int e = 0; e < 4; e++) {
                sh[e] = fmaf(hp[r], w[2 * r + e], sh[e]);
                sl[e] = fmaf(lp[r], w[2 * r + e], sl[e]);
              }
          }
        } else {
#pragma unroll
          for (int r = 0; r < ORDER; r++) {
            const float4 v = *reinterpret_cast<const float4 *>(in + i0 + r * dil);
            const float ve[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
            for (int e = 0; e < 4; e++) {
              sh[e] = fmaf(hp[r], ve[e], sh[e]);
              sl[e] = fmaf(lp[r], ve[e], sl[e]);
            }
          }
        }
        const float4 hv = make_float4(sh[0], sh[1], sh[2], sh[3]);
        const float4 lv = make_float4(sl[0], sl[1], sl[2], sl[3]);
        float4 *hrow = reinterpret_cast<float4 *>(hi + sig * hs + static_cast<int64_t>(l) * len);
        if (NT) {
          typedef float native4 __attribute__((ext_vector_type(4)));
          const native4 nv = {hv.x, hv.y, hv.z, hv.w};
          __builtin_nontemporal_store(nv, reinterpret_cast<native4 *>(hrow + q));
        } else {
          hrow[q] = hv;
        }
        if (last)
          reinterpret_cast<float4 *>(lo + sig * ls)[q] = lv;
        else
          put(out, i0, lv, next_halo);
      }
    }
    par ^= 1;
  }
}

// Signals per workgroup of the fused kernel (vs_tune_set("swt_sigs", 1 / 2)).
extern thread_local int g_swt_sigs;

template <int ORDER, bool NT, int SIGS>
vs_status launch_swt_fused_t(const Taps &t, int ext, int levels, const float *src, int len,
                             float *hi, int64_t hs, float *lo, int64_t ls, int batch,
                             hipStream_t s) {
  const int halo = (ORDER - 1) << (levels - 1);
  const size_t lds =
      2 * SIGS * static_cast<size_t>((len + halo + 2 * ORDER + 8 + 3) & ~3) * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(swt_fused_kernel<ORDER, NT, SIGS>),
      hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  VS_HIP(attr);
  hipLaunchKernelGGL((swt_fused_kernel<ORDER, NT, SIGS>),
                     dim3(static_cast<unsigned>((batch + SIGS - 1) / SIGS)), dim3(256), lds, s, t,
                     ext, levels, src, len, hi, hs, lo, ls, batch);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

template <int ORDER>
vs_status launch_swt_fused(const Taps &t, int ext, int levels, const float *src, int len,
                           float *hi, int64_t hs, float *lo, int64_t ls, int batch, bool nt,
                           hipStream_t s) {
  const int halo = (ORDER - 1) << (levels - 1);
  const size_t one = 2 * static_cast<size_t>((len + halo + 2 * ORDER + 8 + 3) & ~3) * sizeof(float);
  // several signals per workgroup while their bands fit the CU's LDS
  int sigs = std::max(1, std::min(g_swt_sigs, batch));
  while (sigs > 1 && sigs * one > 150 * 1024) sigs--;
#define VS_SWT_SIGS(N)                                                                          \
  case N:                                                                                       \
    return nt ? launch_swt_fused_t<ORDER, true, N>(t, ext, levels, src, len, hi, hs, lo, ls,   \
                                                   batch, s)                                    \
              : launch_swt_fused_t<ORDER, false, N>(t, ext, levels, src, len, hi, hs, lo, ls,  \
                                                    batch, s);
  switch (sigs) {
    VS_SWT_SIGS(5) VS_SWT_SIGS(4) VS_SWT_SIGS(3) VS_SWT_SIGS(2)
    default: break;
  }
  switch (1) { VS_SWT_SIGS(1) }
  return VS_ERR_INVALID;
#undef VS_SWT_SIGS
}

// Signals longer than one workgroup's LDS (len > kMultiMax): tiles of
// kTileOut outputs, each workgroup loading its tile plus the whole multi-level
// support H = (ORDER-1)(2^L - 1) and running every level in LDS.  The band
// of level l covers T + (ORDER-1)(2^L - 2^l) positions, so the last level
// yields exactly the tile.  One HBM pass: read (1 + H/T) x, write L hi rows +
// lo, instead of ~3 passes per level through HBM.
// Positions past the end of the signal: periodic extension is exact by
// circularity (computing a band from the periodic extension of its input gives
// the periodic extension of the band); mirror / constant / zero are re-applied
// to each band by the last tile, which starts at len - T so the mirrored
// samples (the band's last H positions) are in its LDS.
constexpr int kTileOut = 4096;

template <int ORDER>
__global__ __launch_bounds__(256) void swt_tiled_kernel(
    Taps taps, int ext, int levels, const float *__restrict__ src, int64_t len,
    float *__restrict__ hi, int64_t hs, float *__restrict__ lo, int64_t ls) {
  extern __shared__ __attribute__((aligned(16))) float smemt[];
  const int H = (ORDER - 1) * ((1 << levels) - 1);
  const int stride = (kTileOut + H + 2 * ORDER + 16 + 3) & ~3;
  float *in = smemt, *out = smemt + stride;
  const int64_t sig = blockIdx.y;
  const int ntiles = gridDim.x;
  const int64_t t0 = static_cast<int>(blockIdx.x) == ntiles - 1
                         ? len - kTileOut
                         : static_cast<int64_t>(blockIdx.x) * kTileOut;
  const bool tail = t0 + kTileOut + H > len;  // band reaches past the signal
  float hp[ORDER], lp[ORDER];
#pragma unroll
  for (int r = 0; r < ORDER; r++) {
    hp[r] = taps.hp[r];
    lp[r] = taps.lp[r];
  }
  const float *x = src + sig * len;
  for (int i = threadIdx.x; i < stride; i += blockDim.x) {
    const int64_t p = t0 + i;
    in[i] = p < len ? __builtin_nontemporal_load(x + p) : ext_load(x, p, len, ext);
  }
  for (int l = 0; l < levels; l++) {
    const int dil = 1 << l;
    const int nout = (kTileOut + (ORDER - 1) * ((1 << levels) - (2 << l)) + 3) & ~3;
    __syncthreads();
    float4 *hrow = reinterpret_cast<float4 *>(hi + sig * hs + l * len + t0);
    const bool last = l == levels - 1;
    for (int q = threadIdx.x; q < nout / 4; q += blockDim.x) {
      const int i0 = 4 * q;
      float sh[4] = {0.f, 0.f, 0.f, 0.f}, sl[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int r = 0; r < ORDER; r++) {
        float ve[4];
        if (dil >= 4) {
          const float4 v = *reinterpret_cast<const float4 *>(in + i0 + r * dil);
          ve[0] = v.x;
          ve[1] = v.y;
          ve[2] = v.z;
          ve[3] = v.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; e++) ve[e] = in[i0 + r * dil + e];
        }
#pragma unroll
        for (int e = 0; e < 4; e++) {
          sh[e] = fmaf(hp[r], ve[e], sh[e]);
          sl[e] = fmaf(lp[r], ve[e], sl[e]);
        }
      }
      const float4 lv = make_float4(sl[0], sl[1], sl[2], sl[3]);
      if (i0 < kTileOut) {
        typedef float native4 __attribute__((ext_vector_type(4)));
        const native4 nv = {sh[0], sh[1], sh[2], sh[3]};
        __builtin_nontemporal_store(nv, reinterpret_cast<native4 *>(hrow + q));
        if (last) {
          const native4 nl = {lv.x, lv.y, lv.z, lv.w};
          __builtin_nontemporal_store(nl, reinterpret_cast<native4 *>(lo + sig * ls + t0) + q);
        }
      }
      if (!last) reinterpret_cast<float4 *>(out)[q] = lv;
    }
    if (!last && tail && ext != EXTENSION_TYPE_PERIODIC) {
      // re-extend the new band past the end of the signal from its own values
      __syncthreads();
      const int end = static_cast<int>(len - t0);  // local index of position len
      for (int i = end + threadIdx.x; i < nout; i += blockDim.x) {
        const int t = i - end;  // < the tile's support, itself < len
        float v = 0.f;
        if (ext == EXTENSION_TYPE_MIRROR) v = out[end - 1 - t];
        else if (ext == EXTENSION_TYPE_CONSTANT) v = out[end - 1];
        out[i] = v;
      }
    }
    float *tmp = in;
    in = out;
    out = tmp;
  }
}

template <int ORDER>
vs_status launch_swt_tiled(const Taps &t, int ext, int levels, const float *src, int64_t len,
                           float *hi, int64_t hs, float *lo, int64_t ls, int batch,
                           hipStream_t s) {
  const int H = (ORDER - 1) * ((1 << levels) - 1);
  const size_t lds = 2 * static_cast<size_t>((kTileOut + H + 2 * ORDER + 16 + 3) & ~3) * 4;
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(swt_tiled_kernel<ORDER>),
      hipFuncAttributeMaxDynamicSharedMemorySize,
      2 * (kTileOut + kMultiExt + 2 * 30 + 16 + 3) * 4);
  VS_HIP(attr);
  const dim3 grid(static_cast<unsigned>((len + kTileOut - 1) / kTileOut),
                  static_cast<unsigned>(batch));
  hipLaunchKernelGGL(swt_tiled_kernel<ORDER>, grid, dim3(256), lds, s, t, ext, levels, src,
                     len, hi, hs, lo, ls);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// Tuning knobs (vs_tune_set): "swt_fused" 0 = the scalar kernels
// (swt_multi_kernel, level by level for long rows), 1 (default) = the
// fused-extension and tiled kernels; "swt_nt" 1 (default) = non-temporal
// hi stores (+3 % on db8 x 8 levels: the hi rows are never re-read here).
thread_local int g_swt_fused = 1;
thread_local int g_swt_nt = 1;
thread_local int g_swt_sigs = 2;
// "dwt_vec" 1 (default) = vectorised pyramid kernel (dwt_multi4_kernel),
// 0 = the scalar kernel.
thread_local int g_dwt_vec = 1;
// "dwt_threads": workgroup size of the vectorised pyramid (0 = auto).
thread_local int g_dwt_threads = 0;
// Tiled decimated levels (dwt_tiled_kernel): input samples per tile and the
// share of a tile its multi-level support may take (1 / g_dwt_halo_div).
// Measured on 1024 x 65536, 8 levels (profiles/r3/wavelet/dwt_tiled.md): tiles
// of 4096 with support <= 1/16 of the tile (db8: 5 + 3 levels in two passes,
// 27 KB of LDS, 5 workgroups per CU) run db8 at 4.8 TB/s against 3.1 for
// 8192-sample tiles holding all 8 levels (62 KB, 2 workgroups per CU).
constexpr int kDwtTile = 4096;
constexpr int kDwtHaloDiv = 16;
thread_local int g_dwt_tile = kDwtTile, g_dwt_halo_div = kDwtHaloDiv;

// Mallat pyramid of one signal in LDS: out row = [hi_1 | hi_2 | ... | hi_L | lo_L].
constexpr int kDwtMultiMax = 16384;

__global__ __launch_bounds__(1024) void dwt_multi_kernel(
    Taps taps, int ext, int levels, const float *__restrict__ src, int len,
    float *__restrict__ out) {
  __shared__ float band[kDwtMultiMax + kMaxOrder + kDwtMultiMax / 2];
  const int64_t sig = blockIdx.x;
  const float *x = src + sig * len;
  float *orow = out + sig * len;
  for (int i = threadIdx.x; i < len; i += blockDim.x) band[i] = x[i];
  __syncthreads();
  int n = len, off = 0;
  float *in = band, *nxt = band + kDwtMultiMax + kMaxOrder;
  for (int l = 0; l < levels; l++) {
    const int half = n / 2;
    for (int t = threadIdx.x; t < taps.order; t += blockDim.x) {
      const int j = ext_index(n + t, n, ext);
      in[n + t] = j < 0 ? 0.f : in[j];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < half; k += blockDim.x) {
      float sh = 0.f, sl = 0.f;
      for (int j = 0; j < taps.order; j++) {
        const float v = in[2 * k + j];
        sh = fmaf(taps.hp[j], v, sh);
        sl = fmaf(taps.lp[j], v, sl);
      }
      orow[off + k] = sh;
      nxt[k] = sl;
    }
    __syncthreads();
    // the new low band becomes the input; copy it to the front half
    for (int k = threadIdx.x; k < half; k += blockDim.x) in[k] = nxt[k];
    __syncthreads();
    off += half;
    n = half;
  }
  for (int k = threadIdx.x; k < n; k += blockDim.x) orow[off + k] = in[k];
}

// Pyramid with compile-time filter length, 256 threads and LDS sized to the
// signal (dynamic): several signals per CU instead of one 98 KB block.
template <int ORDER>
__global__ __launch_bounds__(256) void dwt_multi_t_kernel(
    Taps taps, int ext, int levels, const float *__restrict__ src, int len,
    float *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float dband[];
  float hp[ORDER], lp[ORDER];
#pragma unroll
  for (int r = 0; r < ORDER; r++) {
    hp[r] = taps.hp[r];
    lp[r] = taps.lp[r];
  }
  const int64_t sig = blockIdx.x;
  const float *x = src + sig * len;
  float *orow = out + sig * len;
  float *in = dband, *nxt = dband + len + ORDER;
  for (int i = threadIdx.x; i < len; i += blockDim.x) in[i] = x[i];
  __syncthreads();
  int n = len, off = 0;
  for (int l = 0; l < levels; l++) {
    const int half = n / 2;
    for (int t = threadIdx.x; t < ORDER; t += blockDim.x) {
      const int j = ext_index(n + t, n, ext);
      in[n + t] = j < 0 ? 0.f : in[j];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < half; k += blockDim.x) {
      float sh = 0.f, sl = 0.f;
#pragma unroll
      for (int j = 0; j < ORDER; j++) {
        const float v = in[2 * k + j];
        sh = fmaf(hp[j], v, sh);
        sl = fmaf(lp[j], v, sl);
      }
      orow[off + k] = sh;
      nxt[k] = sl;
    }
    __syncthreads();
    float *t = in;  // the new low band becomes the input
    in = nxt;
    nxt = t;
    off += half;
    n = half;
  }
  for (int k = threadIdx.x; k < n; k += blockDim.x) orow[off + k] = in[k];
}

// Vectorised pyramid: float4 input loads, four consecutive outputs
// per lane from a float4 register window (inputs 2k .. 2k + 6 + ORDER - 1),
// float4 hi stores and low-band writes; the two LDS bands are len and len / 2
// (+ pads) so three 8192-sample workgroups share a CU.  Levels whose half
// length is not a multiple of 4 run the scalar loop.  Measured (65536 x 1024
// / 8192 x 8192, db8, 5 levels): profiles/r2/swt/dwt.md.
template <int ORDER>
__global__ __launch_bounds__(256) void dwt_multi4_kernel(
    Taps taps, int ext, int levels, const float *__restrict__ src, int len,
    float *__restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) float dband4[];
  constexpr int kPad = 16 + ORDER;
  float hp[ORDER], lp[ORDER];
#pragma unroll
  for (int r = 0; r < ORDER; r++) {
    hp[r] = taps.hp[r];
    lp[r] = taps.lp[r];
  }
  const int64_t sig = blockIdx.x;
  const float *x = src + sig * len;
  float *orow = out + sig * len;
  float *bandA = dband4, *bandB = dband4 + ((len + kPad + 3) & ~3);
  for (int q = threadIdx.x; q < len / 4; q += blockDim.x) {
    typedef float native4 __attribute__((ext_vector_type(4)));
    const native4 nv = __builtin_nontemporal_load(reinterpret_cast<const native4 *>(x) + q);
    reinterpret_cast<float4 *>(bandA)[q] = make_float4(nv.x, nv.y, nv.z, nv.w);
  }
  __syncthreads();  // the level-0 extension reads samples other lanes loaded
  float *in = bandA, *nxt = bandB;
  int n = len, off = 0;
  for (int l = 0; l < levels; l++) {
    const int half = n / 2;
    for (int t = threadIdx.x; t < ORDER; t += blockDim.x) {
      const int j = ext_index(n + t, n, ext);
      in[n + t] = j < 0 ? 0.f : in[j];
    }
    __syncthreads();
    if (half % 4 == 0) {
      constexpr int W = (6 + ORDER + 3) / 4;  // float4 window per 4 outputs
      for (int q = threadIdx.x; q < half / 4; q += blockDim.x) {
        float w[4 * W];
#pragma unroll
        for (int c = 0; c < W; c++) {
          const float4 v = reinterpret_cast<const float4 *>(in + 8 * q)[c];
          w[4 * c] = v.x;
          w[4 * c + 1] = v.y;
          w[4 * c + 2] = v.z;
          w[4 * c + 3] = v.w;
        }
        float sh[4] = {0.f, 0.f, 0.f, 0.f}, sl[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < ORDER; j++)
#pragma unroll
          for (int e = 0; e < 4; e++) {
            sh[e] = fmaf(hp[j], w[2 * e + j], sh[e]);
            sl[e] = fmaf(lp[j], w[2 * e + j], sl[e]);
          }
        {
          typedef float native4 __attribute__((ext_vector_type(4)));
          const native4 nv = {sh[0], sh[1], sh[2], sh[3]};
          __builtin_nontemporal_store(nv, reinterpret_cast<native4 *>(orow + off) + q);
        }
        reinterpret_cast<float4 *>(nxt)[q] = make_float4(sl[0], sl[1], sl[2], sl[3]);
      }
    } else {
      for (int k = threadIdx.x; k < half; k += blockDim.x) {
        float sh = 0.f, sl = 0.f;
#pragma unroll
        for (int j = 0; j < ORDER; j++) {
          const float v = in[2 * k + j];
          sh = fmaf(hp[j], v, sh);
          sl = fmaf(lp[j], v, sl);
        }
        orow[off + k] = sh;
        nxt[k] = sl;
      }
    }
    __syncthreads();
    float *t = in;  // the new low band becomes the input
    in = nxt;
    nxt = t;
    off += half;
    n = half;
  }
  for (int k = threadIdx.x; k < n; k += blockDim.x) orow[off + k] = in[k];
}

template <int ORDER>
vs_status launch_dwt_multi4(const Taps &t, int ext, int levels, const float *src, int len,
                            float *out, int batch, hipStream_t s) {
  constexpr int kPad = 16 + ORDER;
  const size_t lds = (((len + kPad + 3) & ~3) + len / 2 + kPad) * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(dwt_multi4_kernel<ORDER>),
      hipFuncAttributeMaxDynamicSharedMemorySize,
      (((kDwtMultiMax + kPad + 3) & ~3) + kDwtMultiMax / 2 + kPad) * 4);
  VS_HIP(attr);
  // About 16 samples per lane (two quads at level 0): 1024-sample signals
  // run 64-lane workgroups (+31 % db2, +48 % db8 over 256 lanes), 8192 and
  // longer 256 (profiles/r2/swt/dwt.md).
  int threads = std::min(256, std::max(64, (len / 16 + 63) / 64 * 64));
  if (g_dwt_threads >= 64 && g_dwt_threads <= 256 && g_dwt_threads % 64 == 0)
    threads = g_dwt_threads;
  hipLaunchKernelGGL(dwt_multi4_kernel<ORDER>, dim3(static_cast<unsigned>(batch)), dim3(threads),
                     lds, s, t, ext, levels, src, len, out);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// Decimated levels on signals of any length: tiles of `tile` input samples
// (a multiple of 2^levels) plus the whole multi-level support
// H = (ORDER-1)(2^levels - 1); every level runs in LDS, level l's band
// covering tile / 2^l + (ORDER-1)(2^(levels-l) - 1) positions, so the last
// level yields exactly tile / 2^levels outputs.  One pass over HBM: each hi
// band goes straight to its place in the output row (a pyramid row, or the
// hi array of a single level), the last low band to `lo`.  float4 window
// reads, four outputs per lane, non-temporal float4 hi stores.
// Past the end of a band: the periodic extension is exact by circularity
// (band lengths are even); mirror / constant / zero are re-applied to each
// new band from its own last values, which the tile that reaches the end
// holds (the last tile starts at len - tile; host: support <= tile / 4 at most).
struct DwtTileArgs {
  const float *src;
  int64_t ss, len;       // row stride and length of the input band
  float *hi;
  int64_t hs, hoff;      // hi of level l at hi + row hs + hoff + sum_{i<l} len / 2^(i+1)
  float *lo;
  int64_t ls;            // last level's low band at lo + row ls
  int levels, ext, tile;
  int vin, vout;         // 16-byte aligned input rows / output segments
  int ntload;            // non-temporal input loads
};


template <int ORDER>
__global__ __launch_bounds__(256) void dwt_tiled_kernel(Taps taps, DwtTileArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smemd[];
  const int L = a.levels, T0 = a.tile;
  const int H0 = (ORDER - 1) * ((1 << L) - 1);
  const int sizeA = (T0 + H0 + 16 + 3) & ~3;
  float *in = smemd, *out = smemd + sizeA;
  const int64_t sig = blockIdx.y;
  const int64_t t0 = blockIdx.x == gridDim.x - 1 ? a.len - T0
                                                  : static_cast<int64_t>(blockIdx.x) * T0;
  float hp[ORDER], lp[ORDER];
#pragma unroll
  for (int r = 0; r < ORDER; r++) {
    hp[r] = taps.hp[r];
    lp[r] = taps.lp[r];
  }
  const float *x = a.src + sig * a.ss;
  const int nin = T0 + H0;
  for (int i = 4 * threadIdx.x; i < sizeA; i += 4 * blockDim.x) {
    const int64_t p = t0 + i;
    float4 v;
    if (a.vin && p + 3 < a.len) {
      if (a.ntload) {
        typedef float native4 __attribute__((ext_vector_type(4)));
        const native4 nv = __builtin_nontemporal_load(reinterpret_cast<const native4 *>(x + p));
        v = make_float4(nv.x, nv.y, nv.z, nv.w);
      } else {
        v = *reinterpret_cast<const float4 *>(x + p);
      }
    } else {
      v.x = i < nin ? ext_load(x, p, a.len, a.ext) : 0.f;
      v.y = i + 1 < nin ? ext_load(x, p + 1, a.len, a.ext) : 0.f;
      v.z = i + 2 < nin ? ext_load(x, p + 2, a.len, a.ext) : 0.f;
      v.w = i + 3 < nin ? ext_load(x, p + 3, a.len, a.ext) : 0.f;
    }
    *reinterpret_cast<float4 *>(in + i) = v;
  }
  int64_t n = a.len, hoff = a.hoff;
  int T = T0;
  for (int l = 0; l < L; l++) {
    const int Tn = T >> 1;                                      // the tile's own outputs
    const int Hn = (ORDER - 1) * ((1 << (L - l - 1)) - 1);      // support of the levels left
    const int nout = (Tn + Hn + 3) & ~3;
    const int64_t nn = n >> 1;
    const int64_t k0 = t0 >> (l + 1);
    const bool last = l == L - 1;
    lds_barrier();
    float *hrow = a.hi + sig * a.hs + hoff + k0;
    float *lrow = a.lo + sig * a.ls + k0;
    if (a.vout && (Tn & 3) == 0 && (nn & 3) == 0) {
      constexpr int W = (6 + ORDER + 3) / 4;  // float4 window of 4 outputs
      for (int q = threadIdx.x; q < nout / 4; q += blockDim.x) {
        float w[4 * W];
#pragma unroll
        for (int c = 0; c < W; c++) {
          const float4 v = reinterpret_cast<const float4 *>(in + 8 * q)[c];
          w[4 * c] = v.x;
          w[4 * c + 1] = v.y;
          w[4 * c + 2] = v.z;
          w[4 * c + 3] = v.w;
        }
        float sh[4] = {0.f, 0.f, 0.f, 0.f}, sl[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < ORDER; j++)
#pragma unroll
          for (int e = 0; e < 4; e++) {
            sh[e] = fmaf(hp[j], w[2 * e + j], sh[e]);
            sl[e] = fmaf(lp[j], w[2 * e + j], sl[e]);
          }
        const float4 lv = make_float4(sl[0], sl[1], sl[2], sl[3]);
        if (4 * q < Tn) {
          typedef float native4 __attribute__((ext_vector_type(4)));
          const native4 nv = {sh[0], sh[1], sh[2], sh[3]};
          __builtin_nontemporal_store(nv, reinterpret_cast<native4 *>(hrow) + q);
          if (last) reinterpret_cast<float4 *>(lrow)[q] = lv;
        }
        if (!last) reinterpret_cast<float4 *>(out)[q] = lv;
      }
    } else {
      for (int k = threadIdx.x; k < Tn + Hn; k += blockDim.x) {
        float sh = 0.f, sl = 0.f;
#pragma unroll
        for (int j = 0; j < ORDER; j++) {
          const float v = in[2 * k + j];
          sh = fmaf(hp[j], v, sh);
          sl = fmaf(lp[j], v, sl);
        }
        if (k < Tn) {
          hrow[k] = sh;
          if (last) lrow[k] = sl;
        }
        if (!last) out[k] = sl;
      }
    }
    if (!last && a.ext != EXTENSION_TYPE_PERIODIC && k0 + nout > nn) {
      // re-extend the new band past its end from its own values
      lds_barrier();
      const int end = static_cast<int>(nn - k0);  // local index of position nn
      for (int i = end + threadIdx.x; i < nout; i += blockDim.x) {
        const int64_t t = i - end;
        float v = 0.f;
        if (a.ext == EXTENSION_TYPE_MIRROR) v = out[end - 1 - static_cast<int>(t % nn)];
        else if (a.ext == EXTENSION_TYPE_CONSTANT) v = out[end - 1];
        out[i] = v;
      }
    }
    float *tmp = in;
    in = out;
    out = tmp;
    n = nn;
    hoff += nn;
    T = Tn;
  }
}

// Levels one tiled pass can fuse: their support must fit 1 / g_dwt_halo_div
// (at most a quarter) of the tile, so every tile that reaches the end of a
// band holds the samples its re-extension mirrors and the halo work stays
// small.
inline int dwt_tile_levels(int order, int64_t tile, int want) {
  int l = 1;
  while (l < want && static_cast<int64_t>(order - 1) * ((2LL << l) - 1) <= tile / g_dwt_halo_div)
    l++;
  return l;
}

template <int ORDER>
vs_status launch_dwt_tiled(const Taps &t, DwtTileArgs a, int batch, hipStream_t s) {
  a.tile = static_cast<int>(std::min<int64_t>(g_dwt_tile, a.len));
  const int H0 = (ORDER - 1) * ((1 << a.levels) - 1);
  const int H1 = (ORDER - 1) * ((1 << (a.levels - 1)) - 1);
  const size_t lds = (static_cast<size_t>((a.tile + H0 + 16 + 3) & ~3) +
                      static_cast<size_t>((a.tile / 2 + H1 + 16 + 3) & ~3)) * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(dwt_tiled_kernel<ORDER>),
      hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
  VS_HIP(attr);
  VS_REQUIRE(lds <= 96 * 1024, "dwt: tile of %d samples x %d levels needs %zu bytes of LDS",
             a.tile, a.levels, lds);
  const auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  a.vin = al(a.src) && a.ss % 4 == 0 && a.len % 4 == 0 && a.tile % 4 == 0;
  a.vout = al(a.hi) && al(a.lo) && a.hs % 4 == 0 && a.ls % 4 == 0 && a.hoff % 4 == 0;
  // single levels stream their input once (5.5 -> 5.8-6.0 TB/s with
  // non-temporal loads); the multi-level passes measured level either way
  a.ntload = a.levels == 1;
  const int threads = std::min(256, std::max(64, (a.tile / 16 + 63) / 64 * 64));
  const dim3 grid(static_cast<unsigned>((a.len + a.tile - 1) / a.tile),
                  static_cast<unsigned>(batch));
  hipLaunchKernelGGL(dwt_tiled_kernel<ORDER>, grid, dim3(threads), lds, s, t, a);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// false: no instantiation for this filter length (callers fall back).
bool dwt_tiled(const Taps &t, const DwtTileArgs &a, int batch, hipStream_t s, vs_status *st) {
  switch (t.order) {
#define VS_DWT_TILED(O) \
  case O: *st = launch_dwt_tiled<O>(t, a, batch, s); return true;
    VS_DWT_TILED(2) VS_DWT_TILED(4) VS_DWT_TILED(6) VS_DWT_TILED(8) VS_DWT_TILED(10)
    VS_DWT_TILED(12) VS_DWT_TILED(14) VS_DWT_TILED(16) VS_DWT_TILED(18) VS_DWT_TILED(20)
    VS_DWT_TILED(24) VS_DWT_TILED(30)
#undef VS_DWT_TILED
    default: return false;
  }
}

template <int ORDER>
vs_status launch_dwt_multi_t(const Taps &t, int ext, int levels, const float *src, int len,
                             float *out, int batch, hipStream_t s) {
  const size_t lds = (2 * static_cast<size_t>(len) + 2 * ORDER) * sizeof(float);
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(dwt_multi_t_kernel<ORDER>),
      hipFuncAttributeMaxDynamicSharedMemorySize, (2 * kDwtMultiMax + 2 * 76) * 4);
  VS_HIP(attr);
  hipLaunchKernelGGL(dwt_multi_t_kernel<ORDER>, dim3(static_cast<unsigned>(batch)), dim3(256),
                     lds, s, t, ext, levels, src, len, out);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status launch_swt(const Taps &t, int level, int ext, const float *src,
                     int64_t len, int64_t ss, float *hi, int64_t hs, float *lo,
                     int64_t ls, int batch, hipStream_t s) {
  const int dil = 1 << (level - 1);
  const long long window = kTile + static_cast<long long>(t.order - 1) * dil;
  if (window <= kSwtLds) {
    const dim3 grid(static_cast<unsigned>((len + kTile - 1) / kTile),
                    static_cast<unsigned>(batch));
    hipLaunchKernelGGL(swt_kernel, grid, dim3(kThreads), 0, s, t, ext, dil, src, len,
                       ss, hi, hs, lo, ls);
  } else {
    const dim3 grid(static_cast<unsigned>((len + kThreads - 1) / kThreads),
                    static_cast<unsigned>(batch));
    hipLaunchKernelGGL(swt_global_kernel, grid, dim3(kThreads), 0, s, t, ext, dil,
                       src, len, ss, hi, hs, lo, ls);
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status make_taps(int type, int order, Taps *t) {
  const auto wt = static_cast<WaveletType>(type);
  const float *lp = wavelet_tables::lowpass_f(wt, order);
  VS_REQUIRE(lp, "wavelet: unsupported (type %d, order %d)", type, order);
  t->order = order;
  wavelet_tables::make_filters(lp, order, t->hp, t->lp);
  return VS_OK;
}

}  // namespace

bool tune(const char *key, int value) {
  if (std::strcmp(key, "swt_fused") == 0) {
    g_swt_fused = value < 0 ? 1 : value;
    return true;
  }
  if (std::strcmp(key, "swt_sigs") == 0) {
    g_swt_sigs = value < 0 ? 2 : value;
    return true;
  }
  if (std::strcmp(key, "swt_nt") == 0) {
    g_swt_nt = value < 0 ? 1 : value;
    return true;
  }
  if (std::strcmp(key, "dwt_vec") == 0) {
    g_dwt_vec = value < 0 ? 1 : value;
    return true;
  }
  if (std::strcmp(key, "dwt_tile") == 0) {
    // a multiple of 2^levels per pass: powers of two from 256 to 8192
    if (value >= 0 && (value < 256 || value > 8192 || (value & (value - 1)))) return false;
    g_dwt_tile = value < 0 ? kDwtTile : value;
    return true;
  }
  if (std::strcmp(key, "dwt_halo_div") == 0) {
    g_dwt_halo_div = value < 0 ? kDwtHaloDiv : std::max(value, 4);
    return true;
  }
  if (std::strcmp(key, "dwt_threads") == 0) {
    g_dwt_threads = value < 0 ? 0 : value;
    return true;
  }
  return false;
}

void tune_reset() {
  g_swt_fused = 1;
  g_swt_nt = 1;
  g_swt_sigs = 2;
  g_dwt_vec = 1;
  g_dwt_threads = 0;
  g_dwt_tile = kDwtTile;
  g_dwt_halo_div = kDwtHaloDiv;
}

}  // namespace wav
}  // namespace vs

using namespace vs;
using namespace vs::wav;

extern "C" {

vs_status vs_wavelet_filter(int type, int order, float *out) {
  VS_REQUIRE(out, "vs_wavelet_filter: null pointer");
  const float *lp = wavelet_tables::lowpass_f(static_cast<WaveletType>(type), order);
  VS_REQUIRE(lp, "vs_wavelet_filter: unsupported (type %d, order %d)", type, order);
  for (int i = 0; i < order; i++) out[i] = lp[i];
  return VS_OK;
}

vs_status vs_dwt(int type, int order, int ext, const float *src, int64_t len,
                 int64_t ss, float *hi, float *lo, int64_t os, int batch,
                 vs_stream_t stream) {
  VS_REQUIRE(src && hi && lo, "vs_dwt: null pointer");
  VS_REQUIRE(len > 0 && len % 2 == 0, "vs_dwt: length %lld must be positive and even",
             static_cast<long long>(len));
  VS_REQUIRE(ext >= 0 && ext <= 3, "vs_dwt: bad extension %d", ext);
  VS_REQUIRE(batch >= 0, "vs_dwt: negative batch");
  if (batch == 0) return VS_OK;
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_dwt(type, order, ext, src + b0 * ss, len, ss, hi + b0 * os, lo + b0 * os, os,
                    nb, stream);
    });
  Taps t;
  VS_TRY(make_taps(type, order, &t));
  auto s = static_cast<hipStream_t>(stream);
  if (g_dwt_vec) {
    DwtTileArgs a{src, ss, len, hi, os, 0, lo, os, 1, ext, 0, 0, 0, 0};
    vs_status st;
    if (dwt_tiled(t, a, batch, s, &st)) return st;
  }
  const dim3 grid(static_cast<unsigned>((len / 2 + kTile - 1) / kTile),
                  static_cast<unsigned>(batch));
  hipLaunchKernelGGL(dwt_kernel, grid, dim3(kThreads), 0, s, t, ext, src, len, ss, hi, lo, os);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_swt(int type, int order, int level, int ext, const float *src,
                 int64_t len, int64_t ss, float *hi, float *lo, int64_t os, int batch,
                 vs_stream_t stream) {
  VS_REQUIRE(src && hi && lo, "vs_swt: null pointer");
  VS_REQUIRE(len > 0, "vs_swt: empty input");
  VS_REQUIRE(level >= 1 && level <= 24, "vs_swt: level %d out of range", level);
  VS_REQUIRE(ext >= 0 && ext <= 3, "vs_swt: bad extension %d", ext);
  VS_REQUIRE(batch >= 0, "vs_swt: negative batch");
  if (batch == 0) return VS_OK;
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_swt(type, order, level, ext, src + b0 * ss, len, ss, hi + b0 * os,
                    lo + b0 * os, os, nb, stream);
    });
  Taps t;
  VS_TRY(make_taps(type, order, &t));
  return launch_swt(t, level, ext, src, len, ss, hi, os, lo, os, batch,
                    static_cast<hipStream_t>(stream));
}

}  // extern "C"

// hi rows of signal b at hi + b hs (level l at + l len), its low band at
// lo + b ls.
static vs_status swt_multilevel(int type, int order, int levels, int ext, const float *src,
                                int64_t len64, float *hi, int64_t hs, float *lo, int64_t ls,
                                int batch, vs_stream_t stream) {
  // whole-signal kernels (len <= kMultiMax) index with int; the tiled and
  // level-by-level paths take the 64-bit length
  const int len = static_cast<int>(std::min<int64_t>(len64, INT32_MAX));
  VS_REQUIRE(src && hi && lo, "vs_swt_multilevel: null pointer");
  VS_REQUIRE(levels >= 1 && levels <= 24, "vs_swt_multilevel: levels out of range");
  VS_REQUIRE(len64 > 0, "vs_swt_multilevel: empty input");
  VS_REQUIRE(batch >= 0, "vs_swt_multilevel: negative batch");
  if (batch == 0) return VS_OK;
  Taps t;
  VS_TRY(make_taps(type, order, &t));
  auto s = static_cast<hipStream_t>(stream);
  const long long halo = static_cast<long long>(order - 1) << (levels - 1);
  if (len <= kMultiMax && halo <= kMultiExt && len % 4 == 0 && g_swt_fused) {
    const bool nt = g_swt_nt != 0;
    switch (order) {
#define VS_SWTF(O) \
  case O: return launch_swt_fused<O>(t, ext, levels, src, len, hi, hs, lo, ls, batch, nt, s);
      VS_SWTF(2) VS_SWTF(4) VS_SWTF(6) VS_SWTF(8) VS_SWTF(10) VS_SWTF(12) VS_SWTF(14)
      VS_SWTF(16) VS_SWTF(18) VS_SWTF(20) VS_SWTF(24) VS_SWTF(30)
#undef VS_SWTF
      default: break;
    }
  }
  if (len <= kMultiMax && halo <= kMultiExt) {
    const size_t lds = 2 * (static_cast<size_t>(len) + halo) * sizeof(float);
    static const hipError_t attr = hipFuncSetAttribute(
        reinterpret_cast<const void *>(swt_multi_kernel),
        hipFuncAttributeMaxDynamicSharedMemorySize, 2 * (kMultiMax + kMultiExt) * 4);
    VS_HIP(attr);
    hipLaunchKernelGGL(swt_multi_kernel, dim3(static_cast<unsigned>(batch)),
                       dim3(256), lds, s, t, ext, levels, src, len, hi, hs, lo, ls);
    VS_HIP(hipGetLastError());
    return VS_OK;
  }
  // Long signals: tiles with the whole multi-level support in LDS.
  const long long support = static_cast<long long>(order - 1) * ((1LL << levels) - 1);
  if (len64 > kMultiMax && len64 % 4 == 0 && support <= kMultiExt && batch <= kMaxGridY &&
      g_swt_fused) {
    switch (order) {
#define VS_SWTT(O) \
  case O: return launch_swt_tiled<O>(t, ext, levels, src, len64, hi, hs, lo, ls, batch, s);
      VS_SWTT(2) VS_SWTT(4) VS_SWTT(6) VS_SWTT(8) VS_SWTT(10) VS_SWTT(12) VS_SWTT(14)
      VS_SWTT(16) VS_SWTT(18) VS_SWTT(20) VS_SWTT(24) VS_SWTT(30)
#undef VS_SWTT
      default: break;
    }
  }
  // Otherwise level by level through HBM (lo of level l feeds level l+1,
  // ping-ponging between two scratch bands; the last level writes lo).
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return swt_multilevel(type, order, levels, ext, src + b0 * len64, len64, hi + b0 * hs, hs,
                            lo + b0 * ls, ls, nb, stream);
    });
  DeviceBuffer tmp;
  const size_t band = static_cast<size_t>(len64) * batch;
  VS_TRY(tmp.alloc(2 * band * sizeof(float), s));
  const float *in = src;
  int64_t in_stride = len64;
  for (int l = 1; l <= levels; l++) {
    const bool last = l == levels;
    float *dst = last ? lo : tmp.as<float>() + (l % 2) * band;
    VS_TRY(launch_swt(t, l, ext, in, len64, l == 1 ? len64 : in_stride, hi + (l - 1) * len64, hs,
                      dst, last ? ls : len64, batch, s));
    in = dst;
    in_stride = last ? ls : len64;
  }
  return VS_OK;
}

extern "C" {

vs_status vs_swt_multilevel(int type, int order, int levels, int ext, const float *src,
                            int64_t len, float *hi, float *lo, int batch, vs_stream_t stream) {
  return swt_multilevel(type, order, levels, ext, src, len, hi, levels * len, lo, len, batch,
                        stream);
}

vs_status vs_swt_multilevel_packed(int type, int order, int levels, int ext, const float *src,
                                   int64_t len, float *out, int batch, vs_stream_t stream) {
  VS_REQUIRE(out, "vs_swt_multilevel_packed: null pointer");
  return swt_multilevel(type, order, levels, ext, src, len, out, (levels + 1) * len,
                        out + levels * len, (levels + 1) * len, batch, stream);
}

vs_status vs_dwt_multilevel(int type, int order, int levels, int ext,
                            const float *src, int64_t len64, float *out, int batch,
                            vs_stream_t stream) {
  VS_REQUIRE(src && out, "vs_dwt_multilevel: null pointer");
  VS_REQUIRE(levels >= 1 && levels <= 30 && len64 > 0 && len64 % (1LL << levels) == 0,
             "vs_dwt_multilevel: length %lld not divisible by 2^%d",
             static_cast<long long>(len64), levels);
  VS_REQUIRE(batch >= 0, "vs_dwt_multilevel: negative batch");
  if (batch == 0) return VS_OK;
  Taps t;
  VS_TRY(make_taps(type, order, &t));
  auto s = static_cast<hipStream_t>(stream);
  if (len64 > kDwtMultiMax) {
    if (batch > kMaxGridY)
      return batch_chunks(batch, [&](long long b0, int nb) {
        return vs_dwt_multilevel(type, order, levels, ext, src + b0 * len64, len64,
                                 out + b0 * len64, nb, stream);
      });
    // Long signals: tiled passes of as many levels as a tile's LDS support
    // allows (db8: 8 levels per pass), each hi band written straight into the
    // pyramid row; between passes the low band goes through a scratch row.
    const size_t rows = static_cast<size_t>(batch);
    DeviceBuffer tmp;
    size_t band = 0;  // floats per scratch band (the first pass's low band, all rows)
    const float *in = src;
    int64_t n = len64, in_stride = len64, off = 0;
    int done = 0, pass = 0;
    while (g_dwt_vec != 0 && done < levels) {
      const int64_t tile = std::min<int64_t>(g_dwt_tile, n);
      const int lf = dwt_tile_levels(order, tile, levels - done);
      const int64_t nout = n >> lf;
      const bool last = done + lf == levels;
      if (!last && !tmp.get()) {  // two scratch bands: pass p reads one, writes the other
        band = rows * static_cast<size_t>(nout);
        VS_TRY(tmp.alloc(2 * band * sizeof(float), s));
      }
      float *lo = last ? out + (len64 - nout) : tmp.as<float>() + (pass & 1) * band;
      DwtTileArgs a{in, in_stride, n, out, len64, off, lo, last ? len64 : nout,
                    lf, ext, 0, 0, 0, 0};
      vs_status st;
      if (!dwt_tiled(t, a, batch, s, &st)) break;  // no instantiation for this filter length
      VS_TRY(st);
      in = lo;
      in_stride = nout;
      off += n - nout;
      n = nout;
      done += lf;
      pass++;
    }
    if (done == levels) return VS_OK;
    // Level by level through HBM (vs_dwt), the band of level l feeding
    // level l + 1; hi bands copied into the pyramid rows.
    VS_REQUIRE(done == 0, "vs_dwt_multilevel: internal error (partial tiled pyramid)");
    VS_REQUIRE(len64 < (1LL << 31), "vs_dwt_multilevel: filter length %d has no tiled kernel "
               "for rows of 2^31 samples or more", order);
    const int len = static_cast<int>(len64);
    DeviceBuffer tmp2;
    VS_TRY(tmp2.alloc(2 * rows * static_cast<size_t>(len) * sizeof(float), s));
    float *hbuf = tmp2.as<float>(), *lbuf[2] = {hbuf + rows * (len / 2),
                                                hbuf + rows * len + rows * (len / 4)};
    in = src;
    int nl = len, offl = 0;
    in_stride = len;
    for (int l = 0; l < levels; l++) {
      const int half = nl / 2;
      float *lo = lbuf[l & 1];
      VS_TRY(vs_dwt(type, order, ext, in, nl, in_stride, hbuf, lo, half, batch, stream));
      VS_HIP(hipMemcpy2DAsync(out + offl, len * sizeof(float), hbuf, half * sizeof(float),
                              half * sizeof(float), rows, hipMemcpyDeviceToDevice, s));
      in = lo;
      in_stride = half;
      offl += half;
      nl = half;
    }
    VS_HIP(hipMemcpy2DAsync(out + offl, len * sizeof(float), in, nl * sizeof(float),
                            nl * sizeof(float), rows, hipMemcpyDeviceToDevice, s));
    return VS_OK;
  }
  const int len = static_cast<int>(len64);
  const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(out)) &
                        15) == 0;
  if (g_dwt_vec && len % 4 == 0 && aligned) {
    switch (order) {
#define VS_DWT_V(O) \
  case O: return launch_dwt_multi4<O>(t, ext, levels, src, len, out, batch, s);
      VS_DWT_V(2) VS_DWT_V(4) VS_DWT_V(6) VS_DWT_V(8) VS_DWT_V(12) VS_DWT_V(16) VS_DWT_V(18)
      VS_DWT_V(20) VS_DWT_V(24) VS_DWT_V(30)
#undef VS_DWT_V
      default: break;
    }
  }
  switch (order) {
#define VS_DWT_T(O) \
  case O: return launch_dwt_multi_t<O>(t, ext, levels, src, len, out, batch, s);
    VS_DWT_T(2) VS_DWT_T(4) VS_DWT_T(6) VS_DWT_T(8) VS_DWT_T(12) VS_DWT_T(16) VS_DWT_T(18)
    VS_DWT_T(20) VS_DWT_T(24) VS_DWT_T(30)
#undef VS_DWT_T
    default: break;
  }
  const int threads = len / 2 >= 1024 ? 1024 : ((len / 2 + 63) / 64) * 64;
  hipLaunchKernelGGL(dwt_multi_kernel, dim3(static_cast<unsigned>(batch)),
                     dim3(threads), 0, static_cast<hipStream_t>(stream), t, ext,
                     levels, src, len, out);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // extern "C"
