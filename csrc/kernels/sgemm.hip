// Exact-fp32 SGEMM on the CDNA4 matrix cores.
//
// gfx950 has no TF32/xf32 path, but it does have an f32-in / f32-accumulate
// MFMA (v_mfma_f32_32x32x2_f32, 64 FLOP/clk/SIMD, bit-exact k-ordered fmaf
// chain) that runs at the full fp32 vector rate while leaving the VALU free
// for addressing and staging (cdna_hip_programming.md §3 'FP32-input MFMA').
//
// Structure (template <BM, BN, BK, WM, WN>; WM x WN waves per workgroup):
//   * each wave owns a (BM/WM) x (BN/WN) output block held as 32 x 32 MFMA
//     accumulators (16 accumulator registers each);
//   * K is walked in BK steps through two LDS buffers laid out k-major
//     ([k][m], [k][n], rows padded by 4 floats), so an MFMA operand is one
//     conflict-free ds_read_b32 per lane (32 consecutive floats per half-wave);
//   * register-staged prefetch: the global loads of tile t+1 are issued before
//     the MFMAs of tile t and written to the other LDS buffer after them
//     (T14 issue-early / write-late), one barrier per K step;
//   * operands stored K-contiguous (A as stored, B for NT) are transposed on
//     the LDS write; MN-contiguous ones (B as stored, A for TN) are copied
//     with 16-byte LDS writes;
//   * ragged M/N/K and unaligned leading dimensions (the reference's
//     299 x 125 x 999 test) use guarded scalar loads on edge tiles only;
//   * block ids are remapped so that neighbouring tiles share an XCD's L2
//     (T1), and blockIdx.z walks the batch of strided-batched calls.
//
// Reference counterpart: src/matrix.c:200-252 (AVX dot-product GEMM with a
// stack-copied B column, no blocking) and :53-80 (scalar).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "csrc/kernels/device.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct GemmArgs {
  int m, n, k;
  float alpha, beta;
  const float *a;
  int64_t lda, stride_a;
  const float *b;
  int64_t ldb, stride_b;
  float *c;
  int64_t ldc, stride_c;
};

template <int BM_, int BN_, int BK_, int WM_, int WN_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_;
  static constexpr int kThreads = 64 * WM * WN;
  static constexpr int TM = BM / WM / 32;  // 32x32 tiles per wave along M
  static constexpr int TN = BN / WN / 32;
  static constexpr int PA = BM + 4;        // LDS pitch of the A tile (floats)
  static constexpr int PB = BN + 4;
  static constexpr int kLdsFloats = 2 * BK * (PA + PB);
  static_assert(TM >= 1 && TN >= 1, "wave tile smaller than one MFMA tile");
};

// Loads this thread's share of one BK x BMN operand tile into registers.
//   KCONTIG: operand stored [mn][k] (k contiguous) -> float4 along k.
//   else   : operand stored [k][mn] (mn contiguous) -> float4 along mn.
template <int BMN, int BK, int THREADS, bool KCONTIG, bool VEC>
struct TileIO {
  static constexpr int kLoads = BMN * BK / 4 / THREADS;
  static_assert(kLoads * 4 * THREADS == BMN * BK, "tile not divisible");

  __device__ static void load(const float *__restrict__ p, int64_t ld, int mn0,
                             int mn_lim, int k0, int k_lim, float4 (&r)[kLoads]) {
#pragma unroll
    for (int l = 0; l < kLoads; l++) {
      const int idx = threadIdx.x + l * THREADS;
      int mn, kk;
      if (KCONTIG) {
        mn = mn0 + idx / (BK / 4);
        kk = k0 + (idx % (BK / 4)) * 4;
      } else {
        kk = k0 + idx / (BMN / 4);
        mn = mn0 + (idx % (BMN / 4)) * 4;
      }
      const float *base = KCONTIG ? p + mn * ld + kk : p + kk * ld + mn;
      const bool full = KCONTIG ? (mn < mn_lim && kk + 3 < k_lim)
                                : (kk < k_lim && mn + 3 < mn_lim);
      if (VEC && full) {
        r[l] = *reinterpret_cast<const float4 *>(base);
      } else {
        float v[4];
#pragma unroll
        for (int c = 0; c < 4; c++) {
          const bool ok = KCONTIG ? (mn < mn_lim && kk + c < k_lim)
                                  : (kk < k_lim && mn + c < mn_lim);
          v[c] = ok ? base[c] : 0.f;
        }
        r[l] = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
  }

  __device__ static void store(float *__restrict__ s, int pitch,
                              const float4 (&r)[kLoads]) {
#pragma unroll
    for (int l = 0; l < kLoads; l++) {
      const int idx = threadIdx.x + l * THREADS;
      if (KCONTIG) {
        const int mn = idx / (BK / 4), kq = (idx % (BK / 4)) * 4;
        s[(kq + 0) * pitch + mn] = r[l].x;
        s[(kq + 1) * pitch + mn] = r[l].y;
        s[(kq + 2) * pitch + mn] = r[l].z;
        s[(kq + 3) * pitch + mn] = r[l].w;
      } else {
        const int kk = idx / (BMN / 4), mn = (idx % (BMN / 4)) * 4;
        *reinterpret_cast<float4 *>(s + kk * pitch + mn) = r[l];
      }
    }
  }
};

// TA / TB: operand stored transposed relative to op().  A is K-contiguous
// unless TA; B is K-contiguous only if TB.
template <class C, bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(C::kThreads) void sgemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float lds[C::kLdsFloats];
  using IOA = TileIO<C::BM, C::BK, C::kThreads, !TA, VEC>;
  using IOB = TileIO<C::BN, C::BK, C::kThreads, TB, VEC>;
  constexpr int BK = C::BK, PA = C::PA, PB = C::PB;
  constexpr int kBuf = BK * (PA + PB);

  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN;
  const unsigned tiles_m = (g.m + C::BM - 1) / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = static_cast<int>(t / tiles_n) * C::BM;
  const int n0 = static_cast<int>(t % tiles_n) * C::BN;

  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *Cp = g.c + blockIdx.z * g.stride_c;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int lrow = lane & 31, lk = lane >> 5;
  const int am = wm * (C::BM / C::WM) + lrow;
  const int bn = wn * (C::BN / C::WN) + lrow;

  floatx16 acc[C::TM][C::TN];
#pragma unroll
  for (int i = 0; i < C::TM; i++)
#pragma unroll
    for (int j = 0; j < C::TN; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  float4 ra[IOA::kLoads], rb[IOB::kLoads];
  const int nk = (g.k + BK - 1) / BK;

  IOA::load(A, g.lda, m0, g.m, 0, g.k, ra);
  IOB::load(B, g.ldb, n0, g.n, 0, g.k, rb);
  IOA::store(lds, PA, ra);
  IOB::store(lds + BK * PA, PB, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      IOA::load(A, g.lda, m0, g.m, (kt + 1) * BK, g.k, ra);
      IOB::load(B, g.ldb, n0, g.n, (kt + 1) * BK, g.k, rb);
    }
    const float *As = lds + cur * kBuf;
    const float *Bs = As + BK * PA;
#pragma unroll
    for (int s = 0; s < BK / 2; s++) {
      const int kr = 2 * s + lk;
      float fa[C::TM], fb[C::TN];
#pragma unroll
      for (int i = 0; i < C::TM; i++) fa[i] = As[kr * PA + am + i * 32];
#pragma unroll
      for (int j = 0; j < C::TN; j++) fb[j] = Bs[kr * PB + bn + j * 32];
#pragma unroll
      for (int i = 0; i < C::TM; i++)
#pragma unroll
        for (int j = 0; j < C::TN; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j],
                                                           acc[i][j], 0, 0, 0);
    }
    if (more) {
      float *Ad = lds + (cur ^ 1) * kBuf;
      IOA::store(Ad, PA, ra);
      IOB::store(Ad + BK * PA, PB, rb);
    }
    __syncthreads();
  }

  // Epilogue: C/D map of the 32x32 f32 MFMA: col = lane & 31,
  // row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
  const bool use_beta = g.beta != 0.f;
#pragma unroll
  for (int i = 0; i < C::TM; i++)
#pragma unroll
    for (int j = 0; j < C::TN; j++) {
      const int col = n0 + bn + j * 32;
      if (col >= g.n) continue;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = m0 + am - lrow + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < g.m) {
          float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
          float v = g.alpha * acc[i][j][r];
          if (use_beta) v += g.beta * *pc;
          *pc = v;
        }
      }
    }
}

// ---------------------------------------------------------------------
// Generation 2: K-contiguous LDS images + 16-byte fragment reads.
//
// Both operand tiles are stored k-contiguous in LDS ([m][k] and [n][k],
// pitch BK + 4 floats: conflict-free ds_read_b128 for 16 consecutive rows).
// The 32x32x2 MFMA consumes two k per instruction (lane half h gets one);
// since the order of the K sum is free, MFMA s (s = 0..3) of an 8-k group
// takes k = 4h + s, so every lane fetches its 4 k values for 4 MFMAs with
// ONE ds_read_b128 per operand tile (4x fewer LDS instructions than gen 1).
// Fragments of group g+1 are read while the MFMAs of group g run, interior
// tiles use unguarded 16-byte global loads, edge tiles a guarded copy of the
// same loop (uniform branch per workgroup).
template <int BM_, int BN_, int BK_, int WM_, int WN_>
struct Cfg2 {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_;
  static constexpr int kThreads = 64 * WM * WN;
  static constexpr int TM = BM / WM / 32;
  static constexpr int TN = BN / WN / 32;
  static constexpr int P = BK + 4;  // LDS pitch (floats) of both images
  static constexpr int kBuf = (BM + BN) * P;
  static constexpr int kLdsFloats = 2 * kBuf;
  static_assert(BK % 8 == 0, "BK must be a multiple of 8");
};

// Stage one operand tile (BMN rows of the op, BK deep) into registers.
//   KC: stored [mn][k] (k contiguous)  -> float4 along k, no transpose.
//   else: stored [k][mn]               -> float4 along mn, transposed on store.
template <int BMN, int BK, int THREADS, bool KC>
struct TileIO2 {
  static constexpr int kLoads = BMN * BK / 4 / THREADS;
  static_assert(kLoads * 4 * THREADS == BMN * BK, "tile not divisible");

  template <bool GUARD>
  __device__ static void load(const float *__restrict__ p, int64_t ld, int mn0,
                             int mn_lim, int k0, int k_lim, bool vec,
                             float4 (&r)[kLoads]) {
#pragma unroll
    for (int l = 0; l < kLoads; l++) {
      const int idx = threadIdx.x + l * THREADS;
      int mn, kk;
      if (KC) {
        mn = mn0 + idx / (BK / 4);
        kk = k0 + (idx % (BK / 4)) * 4;
      } else {
        kk = k0 + idx / (BMN / 4);
        mn = mn0 + (idx % (BMN / 4)) * 4;
      }
      const float *base = KC ? p + mn * ld + kk : p + kk * ld + mn;
      if (!GUARD) {
        r[l] = *reinterpret_cast<const float4 *>(base);
      } else {
        const bool full = KC ? (mn < mn_lim && kk + 3 < k_lim)
                             : (kk < k_lim && mn + 3 < mn_lim);
        if (vec && full) {
          r[l] = *reinterpret_cast<const float4 *>(base);
        } else {
          float v[4];
#pragma unroll
          for (int c = 0; c < 4; c++) {
            const bool ok = KC ? (mn < mn_lim && kk + c < k_lim)
                               : (kk < k_lim && mn + c < mn_lim);
            v[c] = ok ? base[c] : 0.f;
          }
          r[l] = make_float4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  }

  // Image layout [mn][k], pitch P.
  template <int P>
  __device__ static void store(float *__restrict__ s, const float4 (&r)[kLoads]) {
#pragma unroll
    for (int l = 0; l < kLoads; l++) {
      const int idx = threadIdx.x + l * THREADS;
      if (KC) {
        const int mn = idx / (BK / 4), kq = (idx % (BK / 4)) * 4;
        *reinterpret_cast<float4 *>(s + mn * P + kq) = r[l];
      } else {
        const int kk = idx / (BMN / 4), mn = (idx % (BMN / 4)) * 4;
        s[(mn + 0) * P + kk] = r[l].x;
        s[(mn + 1) * P + kk] = r[l].y;
        s[(mn + 2) * P + kk] = r[l].z;
        s[(mn + 3) * P + kk] = r[l].w;
      }
    }
  }
};

template <class C, bool TA, bool TB, bool GUARD>
__device__ __forceinline__ void sgemm2_body(const GemmArgs &g, float *lds,
                                            const float *A, const float *B,
                                            float *Cp, int m0, int n0, bool vec) {
  using IOA = TileIO2<C::BM, C::BK, C::kThreads, !TA>;
  using IOB = TileIO2<C::BN, C::BK, C::kThreads, TB>;
  constexpr int BK = C::BK, P = C::P, TM = C::TM, TN = C::TN;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int lrow = lane & 31, lh = lane >> 5;
  const int arow = wm * (C::BM / C::WM) + lrow;
  const int brow = wn * (C::BN / C::WN) + lrow;

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  float4 ra[IOA::kLoads], rb[IOB::kLoads];
  const int nk = (g.k + BK - 1) / BK;
  IOA::template load<GUARD>(A, g.lda, m0, g.m, 0, g.k, vec, ra);
  IOB::template load<GUARD>(B, g.ldb, n0, g.n, 0, g.k, vec, rb);
  IOA::template store<P>(lds, ra);
  IOB::template store<P>(lds + C::BM * P, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      IOA::template load<GUARD>(A, g.lda, m0, g.m, (kt + 1) * BK, g.k, vec, ra);
      IOB::template load<GUARD>(B, g.ldb, n0, g.n, (kt + 1) * BK, g.k, vec, rb);
    }
    const float *As = lds + cur * C::kBuf;
    const float *Bs = As + C::BM * P;
    float4 fa[TM], fb[TN], na[TM], nb[TN];
#pragma unroll
    for (int i = 0; i < TM; i++)
      fa[i] = *reinterpret_cast<const float4 *>(As + (arow + 32 * i) * P + 4 * lh);
#pragma unroll
    for (int j = 0; j < TN; j++)
      fb[j] = *reinterpret_cast<const float4 *>(Bs + (brow + 32 * j) * P + 4 * lh);
#pragma unroll
    for (int gk = 0; gk < BK / 8; gk++) {
      if (gk + 1 < BK / 8) {
        const int ko = 8 * (gk + 1) + 4 * lh;
#pragma unroll
        for (int i = 0; i < TM; i++)
          na[i] = *reinterpret_cast<const float4 *>(As + (arow + 32 * i) * P + ko);
#pragma unroll
        for (int j = 0; j < TN; j++)
          nb[j] = *reinterpret_cast<const float4 *>(Bs + (brow + 32 * j) * P + ko);
      }
#pragma unroll
      for (int sidx = 0; sidx < 4; sidx++)
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
          for (int j = 0; j < TN; j++) {
            const float av = sidx == 0 ? fa[i].x : sidx == 1 ? fa[i].y : sidx == 2 ? fa[i].z : fa[i].w;
            const float bv = sidx == 0 ? fb[j].x : sidx == 1 ? fb[j].y : sidx == 2 ? fb[j].z : fb[j].w;
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[i][j], 0, 0, 0);
          }
      if (gk + 1 < BK / 8) {
#pragma unroll
        for (int i = 0; i < TM; i++) fa[i] = na[i];
#pragma unroll
        for (int j = 0; j < TN; j++) fb[j] = nb[j];
      }
    }
    if (more) {
      float *Ad = lds + (cur ^ 1) * C::kBuf;
      IOA::template store<P>(Ad, ra);
      IOB::template store<P>(Ad + C::BM * P, rb);
    }
    __syncthreads();
  }

  const bool use_beta = g.beta != 0.f;
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++) {
      const int col = n0 + brow + j * 32;
      if (GUARD && col >= g.n) continue;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = m0 + arow - lrow + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (!GUARD || row < g.m) {
          float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
          float v = g.alpha * acc[i][j][r];
          if (use_beta) v += g.beta * *pc;
          *pc = v;
        }
      }
    }
}

template <class C, bool TA, bool TB>
__global__ __launch_bounds__(C::kThreads) void sgemm2_kernel(GemmArgs g, int vec) {
  __shared__ __attribute__((aligned(16))) float lds[C::kLdsFloats];
  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN;
  const unsigned tiles_m = (g.m + C::BM - 1) / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int m0 = static_cast<int>(t / tiles_n) * C::BM;
  const int n0 = static_cast<int>(t % tiles_n) * C::BN;
  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *Cp = g.c + blockIdx.z * g.stride_c;
  const bool interior = vec && m0 + C::BM <= g.m && n0 + C::BN <= g.n &&
                        g.k % C::BK == 0;
  if (interior)
    sgemm2_body<C, TA, TB, false>(g, lds, A, B, Cp, m0, n0, true);
  else
    sgemm2_body<C, TA, TB, true>(g, lds, A, B, Cp, m0, n0, vec != 0);
}

template <class C>
void launch_cfg2(const GemmArgs &g, int ta, int tb, bool vec, int batch,
                 hipStream_t s) {
  const unsigned tiles = static_cast<unsigned>(((g.m + C::BM - 1) / C::BM) *
                                               ((g.n + C::BN - 1) / C::BN));
  const dim3 grid(tiles, 1, static_cast<unsigned>(batch)), block(C::kThreads);
  const int v = vec ? 1 : 0;
  if (!ta && !tb)
    hipLaunchKernelGGL((sgemm2_kernel<C, false, false>), grid, block, 0, s, g, v);
  else if (!ta && tb)
    hipLaunchKernelGGL((sgemm2_kernel<C, false, true>), grid, block, 0, s, g, v);
  else if (ta && !tb)
    hipLaunchKernelGGL((sgemm2_kernel<C, true, false>), grid, block, 0, s, g, v);
  else
    hipLaunchKernelGGL((sgemm2_kernel<C, true, true>), grid, block, 0, s, g, v);
}

template <class C>
void launch_cfg(const GemmArgs &g, int ta, int tb, bool vec, int batch,
                hipStream_t s) {
  const unsigned tiles = static_cast<unsigned>(((g.m + C::BM - 1) / C::BM) *
                                               ((g.n + C::BN - 1) / C::BN));
  const dim3 grid(tiles, 1, static_cast<unsigned>(batch)), block(C::kThreads);
#define VS_L(TA_, TB_)                                                       \
  if (vec)                                                                   \
    hipLaunchKernelGGL((sgemm_kernel<C, TA_, TB_, true>), grid, block, 0, s, g); \
  else                                                                       \
    hipLaunchKernelGGL((sgemm_kernel<C, TA_, TB_, false>), grid, block, 0, s, g);
  if (!ta && !tb) {
    VS_L(false, false)
  } else if (!ta && tb) {
    VS_L(false, true)
  } else if (ta && !tb) {
    VS_L(true, false)
  } else {
    VS_L(true, true)
  }
#undef VS_L
}

// Tile variants (A/B-benchmarked on MI355X, see profiles/).
using CfgSmall = Cfg<64, 64, 32, 2, 2>;     // small / skinny problems
using CfgA = Cfg<128, 128, 16, 2, 2>;
using CfgB = Cfg<128, 128, 32, 2, 2>;
using CfgC = Cfg<256, 128, 16, 4, 2>;
using CfgD = Cfg<128, 256, 16, 2, 4>;
using Cfg2A = Cfg2<128, 128, 32, 2, 2>;
using Cfg2B = Cfg2<128, 256, 32, 2, 4>;
using Cfg2C = Cfg2<256, 128, 32, 4, 2>;
using Cfg2D = Cfg2<128, 128, 64, 2, 2>;

int default_variant() {
  static const int v = [] {
    const char *e = std::getenv("VELES_SGEMM_VARIANT");
    return e && *e ? std::atoi(e) : -1;
  }();
  return v;
}

vs_status sgemm_impl(int variant, int ta, int tb, int m, int n, int k,
                     float alpha, const float *a, int64_t lda, int64_t sa,
                     const float *b, int64_t ldb, int64_t sb, float beta,
                     float *c, int64_t ldc, int64_t sc, int batch,
                     hipStream_t s) {
  VS_REQUIRE(m >= 0 && n >= 0 && k >= 0 && batch >= 0,
             "vs_sgemm: negative dimension");
  if (m == 0 || n == 0 || batch == 0) return VS_OK;
  VS_REQUIRE(a && b && c, "vs_sgemm: null pointer");
  VS_REQUIRE(ldc >= n, "vs_sgemm: ldc (%lld) < n (%d)", (long long)ldc, n);
  VS_REQUIRE(lda >= (ta ? m : k) && ldb >= (tb ? k : n),
             "vs_sgemm: leading dimension too small");
  VS_REQUIRE(batch <= 65535, "vs_sgemm: batch > 65535");
  GemmArgs g{m, n, k, alpha, beta, a, lda, sa, b, ldb, sb, c, ldc, sc};
  const auto al = [](const void *p) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  };
  const bool vec = al(a) && al(b) && lda % 4 == 0 && ldb % 4 == 0 &&
                   (batch == 1 || (sa % 4 == 0 && sb % 4 == 0));
  if (variant < 0) variant = default_variant();
  if (variant < 0) {
    // Few 128x128 tiles cannot fill 256 CUs: use 64x64 tiles then.
    // Largest tile that still gives every CU work (A/B on MI355X,
    // profiles/r1/sgemm_variants.json): 128x256 when >= 512 tiles,
    // 128x128 when >= 256, else 64x64.
    const long t128 = static_cast<long>((m + 127) / 128) * ((n + 127) / 128) * batch;
    const long t256 = static_cast<long>((m + 127) / 128) * ((n + 255) / 256) * batch;
    variant = t256 >= 512 ? 4 : (t128 >= 256 ? 1 : 0);
  }
  switch (variant) {
    case 0: launch_cfg<CfgSmall>(g, ta, tb, vec, batch, s); break;
    case 1: launch_cfg<CfgA>(g, ta, tb, vec, batch, s); break;
    case 2: launch_cfg<CfgB>(g, ta, tb, vec, batch, s); break;
    case 3: launch_cfg<CfgC>(g, ta, tb, vec, batch, s); break;
    case 4: launch_cfg<CfgD>(g, ta, tb, vec, batch, s); break;
    case 5: launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s); break;
    case 6: launch_cfg2<Cfg2B>(g, ta, tb, vec, batch, s); break;
    case 7: launch_cfg2<Cfg2C>(g, ta, tb, vec, batch, s); break;
    case 8: launch_cfg2<Cfg2D>(g, ta, tb, vec, batch, s); break;
    default:
      set_error("vs_sgemm: unknown variant %d", variant);
      return VS_ERR_INVALID;
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // namespace
}  // namespace vs

extern "C" {

vs_status vs_sgemm(int ta, int tb, int m, int n, int k, float alpha,
                   const float *a, int64_t lda, const float *b, int64_t ldb,
                   float beta, float *c, int64_t ldc, vs_stream_t stream) {
  return vs::sgemm_impl(-1, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0, beta,
                        c, ldc, 0, 1, static_cast<hipStream_t>(stream));
}

vs_status vs_sgemm_strided_batched(int ta, int tb, int m, int n, int k,
                                   float alpha, const float *a, int64_t lda,
                                   int64_t sa, const float *b, int64_t ldb,
                                   int64_t sb, float beta, float *c,
                                   int64_t ldc, int64_t sc, int batch,
                                   vs_stream_t stream) {
  return vs::sgemm_impl(-1, ta, tb, m, n, k, alpha, a, lda, sa, b, ldb, sb,
                        beta, c, ldc, sc, batch, static_cast<hipStream_t>(stream));
}

// Tuning entry point: run one explicit tile variant (0..4).
vs_status vs_sgemm_variant(int variant, int ta, int tb, int m, int n, int k,
                           float alpha, const float *a, int64_t lda,
                           const float *b, int64_t ldb, float beta, float *c,
                           int64_t ldc, vs_stream_t stream) {
  return vs::sgemm_impl(variant, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0,
                        beta, c, ldc, 0, 1, static_cast<hipStream_t>(stream));
}

}  // extern "C"
