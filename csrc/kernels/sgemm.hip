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
template <int BMN, int BK, int THREADS, bool KCONTIG, bool VEC, bool INTERIOR = false>
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
      if (INTERIOR) {
        r[l] = *reinterpret_cast<const float4 *>(base);
        continue;
      }
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
// INTERIOR (implies VEC): every tile is whole, no load or store is guarded.
template <class C, bool TA, bool TB, bool VEC, bool INTERIOR = false>
__global__ __launch_bounds__(C::kThreads) void sgemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float lds[C::kLdsFloats];
  using IOA = TileIO<C::BM, C::BK, C::kThreads, !TA, VEC, INTERIOR>;
  using IOB = TileIO<C::BN, C::BK, C::kThreads, TB, VEC, INTERIOR>;
  constexpr int BK = C::BK, PA = C::PA, PB = C::PB;
  constexpr int kBuf = BK * (PA + PB);

  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN;
  const unsigned tiles_m = (g.m + C::BM - 1) / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM;
  const int n0 = static_cast<int>(tn) * C::BN;

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
      if (!INTERIOR && col >= g.n) continue;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = m0 + am - lrow + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (INTERIOR || row < g.m) {
          float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
          float v = g.alpha * acc[i][j][r];
          if (use_beta) v += g.beta * *pc;
          *pc = v;
        }
      }
    }
}

// ---------------------------------------------------------------------
// Generation 2: natural-layout LDS images, 16-byte global loads AND stores,
// fragment reads shaped by the operand's layout.
//
// An operand tile is copied to LDS in the layout it has in memory (no
// transposing scalar stores -- those were 16-way bank conflicts on the
// critical path between k-tiles):
//   K-contiguous ([mn][k], pitch BK + 4):  one ds_read_b128 per lane fetches
//     the 4 k values of 4 consecutive MFMAs (conflict-free: the 16-lane
//     groups of ds_read_b128 hit 16 distinct 4-bank groups at pitch BK + 4);
//   MN-contiguous ([k][mn], pitch BMN + 4): four ds_read_b32, 32 consecutive
//     columns per half-wave (conflict-free).
// The 32x32x2 MFMA consumes two k per instruction (lane half h supplies one);
// the K summation order is free, so MFMA s (s = 0..3) of an 8-k group takes
// k = 4h + s.  Fragments of group g+1 are read while the MFMAs of group g run;
// the next k-tile's global loads are issued at the top of the tile and written
// to the other LDS buffer after group SAT, so their latency is covered by the
// first groups and the stores by the remaining ones; one barrier per k-tile.
// Interior tiles run an unguarded copy of the loop (uniform branch per
// workgroup).
template <int BM_, int BN_, int BK_, int WM_, int WN_, int SAT_ = -1,
          int SCHED_ = 0>
struct Cfg2 {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_;
  // 0: compiler schedule; 1: sched_group_barrier interleave.  (Pinning each
  // group's MFMAs between sched_barrier(0) fences was measured 25-45 % slower
  // than either: profiles/r1/sgemm_variants.md.)
  static constexpr int SCHED = SCHED_;
  static constexpr int kThreads = 64 * WM * WN;
  static constexpr int TM = BM / WM / 32;
  static constexpr int TN = BN / WN / 32;
  static constexpr int NG = BK / 8;                    // 8-k groups per tile
  static constexpr int SAT = SAT_ < 0 ? NG - 1 : SAT_;  // store after group
  static_assert(BK % 8 == 0, "BK must be a multiple of 8");
};

template <int BMN, int BK, int THREADS, bool KC>
struct TileIO2 {
  static constexpr int kLoads = BMN * BK / 4 / THREADS;
  static_assert(kLoads * 4 * THREADS == BMN * BK, "tile not divisible");
  static constexpr int P = KC ? BK + 4 : BMN + 4;      // LDS pitch (floats)
  // ds_read instructions per frag(): the four scalar reads of an MN-contiguous
  // image are merged by the compiler into two ds_read2_b32
  static constexpr int kFragReads = KC ? 1 : 2;
  static constexpr int kFloats = KC ? BMN * P : BK * P;

  // Thread's (mn, k) coordinates of float4 number l of the tile.
  __device__ static void coord(int l, int &mn, int &kk) {
    const int idx = threadIdx.x + l * THREADS;
    if (KC) {
      mn = idx / (BK / 4);
      kk = (idx % (BK / 4)) * 4;
    } else {
      kk = idx / (BMN / 4);
      mn = (idx % (BMN / 4)) * 4;
    }
  }

  template <bool GUARD>
  __device__ static void load(const float *__restrict__ p, int64_t ld, int mn0,
                             int mn_lim, int k0, int k_lim, bool vec,
                             float4 (&r)[kLoads]) {
#pragma unroll
    for (int l = 0; l < kLoads; l++) {
      int mn, kk;
      coord(l, mn, kk);
      mn += mn0;
      kk += k0;
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

  __device__ static void store(float *__restrict__ s, const float4 (&r)[kLoads]) {
#pragma unroll
    for (int l = 0; l < kLoads; l++) {
      int mn, kk;
      coord(l, mn, kk);
      *reinterpret_cast<float4 *>(s + (KC ? mn * P + kk : kk * P + mn)) = r[l];
    }
  }

  // The 4 k values (k0 + 0..3) of row/column `mn` of the image.
  __device__ static float4 frag(const float *__restrict__ s, int mn, int k0) {
    if (KC) return *reinterpret_cast<const float4 *>(s + mn * P + k0);
    return make_float4(s[(k0 + 0) * P + mn], s[(k0 + 1) * P + mn],
                       s[(k0 + 2) * P + mn], s[(k0 + 3) * P + mn]);
  }
};

template <class C, bool TA, bool TB>
struct Layout2 {
  using IOA = TileIO2<C::BM, C::BK, C::kThreads, !TA>;
  using IOB = TileIO2<C::BN, C::BK, C::kThreads, TB>;
  static constexpr int kBuf = IOA::kFloats + IOB::kFloats;
  static constexpr int kLdsFloats = 2 * kBuf;
};

__device__ __forceinline__ float comp(const float4 &v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}

// One steady-state k-tile (a next tile exists): straight-line code, so the
// scheduler sees the whole tile as one region and -- with C::SCHED -- the
// sched_group_barrier sequence at the end pins the interleave: the next
// tile's global loads first, then every MFMA followed by at most one of the
// next group's fragment reads (and, after group SAT, the LDS stores).
template <class C, bool TA, bool TB, bool GUARD, bool MORE>
__device__ __forceinline__ void ktile(const GemmArgs &g, float *lds,
                                      const float *A, const float *B, int m0,
                                      int n0, bool vec, int kt,
                                      floatx16 (&acc)[C::TM][C::TN],
                                      float4 (&ra)[Layout2<C, TA, TB>::IOA::kLoads],
                                      float4 (&rb)[Layout2<C, TA, TB>::IOB::kLoads]) {
  using L = Layout2<C, TA, TB>;
  using IOA = typename L::IOA;
  using IOB = typename L::IOB;
  constexpr int BK = C::BK, TM = C::TM, TN = C::TN, NG = C::NG;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int lrow = lane & 31, lh = lane >> 5;
  const int arow = wm * (C::BM / C::WM) + lrow;
  const int brow = wn * (C::BN / C::WN) + lrow;
  const int cur = kt & 1;
  if (MORE) {
    IOA::template load<GUARD>(A, g.lda, m0, g.m, (kt + 1) * BK, g.k, vec, ra);
    IOB::template load<GUARD>(B, g.ldb, n0, g.n, (kt + 1) * BK, g.k, vec, rb);
  }
  const float *As = lds + cur * L::kBuf;
  const float *Bs = As + IOA::kFloats;
  float4 fa[NG][TM], fb[NG][TN];
#pragma unroll
  for (int gk = 0; gk < NG; gk++) {
    const int ko = 8 * gk + 4 * lh;
#pragma unroll
    for (int i = 0; i < TM; i++) fa[gk][i] = IOA::frag(As, arow + 32 * i, ko);
#pragma unroll
    for (int j = 0; j < TN; j++) fb[gk][j] = IOB::frag(Bs, brow + 32 * j, ko);
#pragma unroll
    for (int sidx = 0; sidx < 4; sidx++)
#pragma unroll
      for (int i = 0; i < TM; i++)
#pragma unroll
        for (int j = 0; j < TN; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(
              comp(fa[gk][i], sidx), comp(fb[gk][j], sidx), acc[i][j], 0, 0, 0);
    if (MORE && gk == C::SAT) {
      float *Ad = lds + (cur ^ 1) * L::kBuf;
      IOA::store(Ad, ra);
      IOB::store(Ad + IOA::kFloats, rb);
    }
  }
  if constexpr (C::SCHED == 1) {
    constexpr int kReads = TM * IOA::kFragReads + TN * IOB::kFragReads;
    constexpr int kMfma = 4 * TM * TN;
    constexpr int kWrites = IOA::kLoads + IOB::kLoads;
    if (MORE) __builtin_amdgcn_sched_group_barrier(0x020, IOA::kLoads + IOB::kLoads, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, kReads, 0);  // group 0 fragments
#pragma unroll
    for (int gk = 0; gk < NG; gk++) {
      // MFMAs of group gk, each followed by one read of group gk+1
#pragma unroll
      for (int q = 0; q < kMfma; q++) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (gk + 1 < NG && q < kReads) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if (MORE && gk == C::SAT && q >= kReads && q < kReads + kWrites)
          __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
      }
    }
  }
  __syncthreads();
}

template <class C, bool TA, bool TB, bool GUARD>
__device__ __forceinline__ void sgemm2_body(const GemmArgs &g, float *lds,
                                            const float *A, const float *B,
                                            float *Cp, int m0, int n0, bool vec) {
  using L = Layout2<C, TA, TB>;
  using IOA = typename L::IOA;
  using IOB = typename L::IOB;
  constexpr int BK = C::BK, TM = C::TM, TN = C::TN, NG = C::NG;
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
  IOA::store(lds, ra);
  IOB::store(lds + IOA::kFloats, rb);
  __syncthreads();

  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (!GUARD && more) {
      ktile<C, TA, TB, GUARD, true>(g, lds, A, B, m0, n0, vec, kt, acc, ra, rb);
      continue;
    }
    if (more) {
      IOA::template load<GUARD>(A, g.lda, m0, g.m, (kt + 1) * BK, g.k, vec, ra);
      IOB::template load<GUARD>(B, g.ldb, n0, g.n, (kt + 1) * BK, g.k, vec, rb);
    }
    const float *As = lds + cur * L::kBuf;
    const float *Bs = As + IOA::kFloats;
    float4 fa[TM], fb[TN], na[TM], nb[TN];
#pragma unroll
    for (int i = 0; i < TM; i++) fa[i] = IOA::frag(As, arow + 32 * i, 4 * lh);
#pragma unroll
    for (int j = 0; j < TN; j++) fb[j] = IOB::frag(Bs, brow + 32 * j, 4 * lh);
#pragma unroll
    for (int gk = 0; gk < NG; gk++) {
      if (gk + 1 < NG) {
        const int ko = 8 * (gk + 1) + 4 * lh;
#pragma unroll
        for (int i = 0; i < TM; i++) na[i] = IOA::frag(As, arow + 32 * i, ko);
#pragma unroll
        for (int j = 0; j < TN; j++) nb[j] = IOB::frag(Bs, brow + 32 * j, ko);
      }
#pragma unroll
      for (int sidx = 0; sidx < 4; sidx++)
#pragma unroll
        for (int i = 0; i < TM; i++)
#pragma unroll
          for (int j = 0; j < TN; j++)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                comp(fa[i], sidx), comp(fb[j], sidx), acc[i][j], 0, 0, 0);
      if (gk == C::SAT && more) {
        float *Ad = lds + (cur ^ 1) * L::kBuf;
        IOA::store(Ad, ra);
        IOB::store(Ad + IOA::kFloats, rb);
      }
      if (gk + 1 < NG) {
#pragma unroll
        for (int i = 0; i < TM; i++) fa[i] = na[i];
#pragma unroll
        for (int j = 0; j < TN; j++) fb[j] = nb[j];
      }
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

// INTERIOR: the launcher checked that every tile is whole and 16-byte
// aligned; that instance carries no guarded code at all.
template <class C, bool TA, bool TB, bool INTERIOR>
__global__ __launch_bounds__(C::kThreads) void sgemm2_kernel(GemmArgs g, int vec) {
  __shared__ __attribute__((aligned(16))) float lds[Layout2<C, TA, TB>::kLdsFloats];
  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN;
  const unsigned tiles_m = (g.m + C::BM - 1) / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM;
  const int n0 = static_cast<int>(tn) * C::BN;
  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *Cp = g.c + blockIdx.z * g.stride_c;
  sgemm2_body<C, TA, TB, !INTERIOR>(g, lds, A, B, Cp, m0, n0, vec != 0);
}

template <class C>
void launch_cfg2(const GemmArgs &g, int ta, int tb, bool vec, int batch,
                 hipStream_t s) {
  const unsigned tiles = static_cast<unsigned>(((g.m + C::BM - 1) / C::BM) *
                                               ((g.n + C::BN - 1) / C::BN));
  const dim3 grid(tiles, 1, static_cast<unsigned>(batch)), block(C::kThreads);
  const bool aligned = vec && g.m % C::BM == 0 && g.n % C::BN == 0 && g.k % C::BK == 0;
  const int v = vec ? 1 : 0;
#define VS_LAUNCH2(TA_, TB_)                                                        \
  if (aligned)                                                                      \
    hipLaunchKernelGGL((sgemm2_kernel<C, TA_, TB_, true>), grid, block, 0, s, g, v); \
  else                                                                              \
    hipLaunchKernelGGL((sgemm2_kernel<C, TA_, TB_, false>), grid, block, 0, s, g, v);
  if (!ta && !tb) {
    VS_LAUNCH2(false, false)
  } else if (!ta && tb) {
    VS_LAUNCH2(false, true)
  } else if (ta && !tb) {
    VS_LAUNCH2(true, false)
  } else {
    VS_LAUNCH2(true, true)
  }
#undef VS_LAUNCH2
}

template <class C>
void launch_cfg(const GemmArgs &g, int ta, int tb, bool vec, int batch,
                hipStream_t s) {
  const unsigned tiles = static_cast<unsigned>(((g.m + C::BM - 1) / C::BM) *
                                               ((g.n + C::BN - 1) / C::BN));
  const dim3 grid(tiles, 1, static_cast<unsigned>(batch)), block(C::kThreads);
  const bool interior = vec && g.m % C::BM == 0 && g.n % C::BN == 0 && g.k % C::BK == 0;
#define VS_L(TA_, TB_)                                                       \
  if (interior)                                                              \
    hipLaunchKernelGGL((sgemm_kernel<C, TA_, TB_, true, true>), grid, block, 0, s, g); \
  else if (vec)                                                              \
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
// ---------------------------------------------------------------------
// Generation 3 (NN, whole tiles only): operand tiles staged by LDS-DMA
// (global_load_lds_dwordx4: no VGPR round trip, no staging VALU), two LDS
// stages, next tile's DMA issued before the current tile's MFMAs, one
// vmcnt(0) + barrier per k-tile.  A image [BM][BK] (k-contiguous, 16-byte
// chunks XOR-swizzled by row so that the 16-lane groups of ds_read_b128 hit
// distinct banks; the XOR is applied to the DMA source address and to the
// read), read as one ds_read_b128 per 8-k group with the permuted k order of
// generation 2; B image [BK][BN] as stored (n-contiguous), four ds_read_b32
// per 8-k group (32 consecutive columns per half-wave: conflict-free).
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;

template <int BM_, int BN_, int BK_, int WM_, int WN_>
struct Cfg3 {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_;
  static constexpr int kThreads = 64 * WM * WN, kWaves = WM * WN;
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static constexpr int NC = BK / 4;                 // 16-byte chunks per A row
  static constexpr int RBA = BK * 4;                // A row bytes
  static constexpr int SA = 256 / RBA;              // A rows per 256-byte bank row
  static constexpr int RBB = BN * 4;                // B row bytes
  static constexpr int kImgA = BM * RBA, kImgB = BK * RBB;
  static constexpr int kStage = kImgA + kImgB, kLdsBytes = 2 * kStage;
  static constexpr int kInstrA = kImgA / 1024 / kWaves, kInstrB = kImgB / 1024 / kWaves;
  static_assert(kInstrA * 1024 * kWaves == kImgA && kInstrB * 1024 * kWaves == kImgB,
                "tile not divisible into whole DMA instructions per wave");
  static_assert(RBA <= 1024 && 1024 % RBB == 0 || RBB % 1024 == 0, "row geometry");
};

template <class C>
__device__ __forceinline__ int swz3(int row, int c) {
  return c ^ ((row / C::SA) & (C::NC - 1));
}

template <class C>
__global__ __launch_bounds__(C::kThreads) void sgemm3_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t s3_lds[];
  constexpr int BK = C::BK, TM = C::TM, TN = C::TN;
  const unsigned tiles_n = g.n / C::BN, tiles_m = g.m / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM, n0 = static_cast<int>(tn) * C::BN;
  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *Cp = g.c + blockIdx.z * g.stride_c;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int lrow = lane & 31, lh = lane >> 5;
  const int arow = wm * (C::BM / C::WM) + lrow;
  const int bcol = wn * (C::BN / C::WN) + lrow;

  auto stage = [&](int buf, int k0) {
    uint8_t *ia = s3_lds + buf * C::kStage;
    uint8_t *ib = ia + C::kImgA;
#pragma unroll
    for (int i = 0; i < C::kInstrA; i++) {
      const int j = wid * C::kInstrA + i;
      const int row = j * (1024 / C::RBA) + lane / C::NC;
      const int c = swz3<C>(row, lane % C::NC);
      const float *src = A + static_cast<int64_t>(m0 + row) * g.lda + k0 + 4 * c;
      __builtin_amdgcn_global_load_lds((glob_void_t *)src, (lds_void_t *)(ia + j * 1024), 16,
                                       0, 0);
    }
#pragma unroll
    for (int i = 0; i < C::kInstrB; i++) {
      const int j = wid * C::kInstrB + i;
      const int byte = j * 1024 + lane * 16;       // linear position in the B image
      const int kr = byte / C::RBB, nc = (byte % C::RBB) / 4;
      const float *src = B + static_cast<int64_t>(k0 + kr) * g.ldb + n0 + nc;
      __builtin_amdgcn_global_load_lds((glob_void_t *)src, (lds_void_t *)(ib + j * 1024), 16,
                                       0, 0);
    }
  };

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  const int nk = g.k / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
    const uint8_t *ia = s3_lds + cur * C::kStage;
    const float *ib = reinterpret_cast<const float *>(ia + C::kImgA);
#pragma unroll
    for (int gk = 0; gk < BK / 8; gk++) {
      float4 fa[TM];
      float fb[TN][4];
#pragma unroll
      for (int x = 0; x < TM; x++) {
        const int r = arow + 32 * x;
        fa[x] = *reinterpret_cast<const float4 *>(ia + r * C::RBA +
                                                  swz3<C>(r, 2 * gk + lh) * 16);
      }
#pragma unroll
      for (int y = 0; y < TN; y++)
#pragma unroll
        for (int q = 0; q < 4; q++) fb[y][q] = ib[(8 * gk + 4 * lh + q) * C::BN + bcol + 32 * y];
#pragma unroll
      for (int q = 0; q < 4; q++)
#pragma unroll
        for (int x = 0; x < TM; x++)
#pragma unroll
          for (int y = 0; y < TN; y++)
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(comp(fa[x], q), fb[y][q],
                                                             acc[x][y], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const bool use_beta = g.beta != 0.f;
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = n0 + bcol + 32 * y;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = m0 + arow - lrow + 32 * x + (r & 3) + 8 * (r >> 2) + 4 * lh;
        float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
        float v = g.alpha * acc[x][y][r];
        if (use_beta) v += g.beta * *pc;
        *pc = v;
      }
    }
}

template <class C>
bool launch_cfg3(const GemmArgs &g, int ta, int tb, bool vec, int batch, hipStream_t s) {
  // whole tiles, NN, 16-byte aligned rows only; otherwise the caller falls back
  if (ta || tb || !vec || g.m % C::BM || g.n % C::BN || g.k % C::BK || g.k == 0) return false;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&sgemm3_kernel<C>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, C::kLdsBytes);
  const unsigned tiles = static_cast<unsigned>((g.m / C::BM) * (g.n / C::BN));
  hipLaunchKernelGGL(sgemm3_kernel<C>, dim3(tiles, 1, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), C::kLdsBytes, s, g);
  return true;
}

// Generation 3 with the 16x16x4 f32 MFMA (v_mfma_f32_16x16x4_f32: 32 cycles,
// same FLOP/cycle as 32x32x2; MI355X_MICROARCH.md 'DVFS give-back' item 7:
// the chip can hold a higher clock on one MFMA shape than the other).
// Lane l: A[row l & 15][k = 4 (l >> 4) + s] and B[k = 4 (l >> 4) + s][col l & 15]
// for step s of a 16-k group (the k order is free), so the A fragment of
// four steps is one ds_read_b128 and the B fragment four ds_read_b32.  The B
// image's 16-byte chunks are XOR-swizzled by bit 2 of the row so that the
// two lane quarters of a 32-lane read group (rows k and k + 4) hit disjoint
// banks.  C/D of 16x16x4: col = lane & 15, row = 4 (lane >> 4) + reg.
typedef float floatx4 __attribute__((ext_vector_type(4)));

template <class C>
__device__ __forceinline__ int bswz(int krow) {
  return ((krow >> 2) & 1) << 2;
}

template <class C>
__global__ __launch_bounds__(C::kThreads) void sgemm3x16_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t s316_lds[];
  constexpr int BK = C::BK;
  constexpr int TM = C::BM / C::WM / 16, TN = C::BN / C::WN / 16;
  const unsigned tiles_n = g.n / C::BN, tiles_m = g.m / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM, n0 = static_cast<int>(tn) * C::BN;
  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *Cp = g.c + blockIdx.z * g.stride_c;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l16 = lane & 15, q = lane >> 4;
  const int arow = wm * (C::BM / C::WM) + l16;
  const int bcol = wn * (C::BN / C::WN) + l16;

  auto stage = [&](int buf, int k0) {
    uint8_t *ia = s316_lds + buf * C::kStage;
    uint8_t *ib = ia + C::kImgA;
#pragma unroll
    for (int i = 0; i < C::kInstrA; i++) {
      const int j = wid * C::kInstrA + i;
      const int row = j * (1024 / C::RBA) + lane / C::NC;
      const int c = swz3<C>(row, lane % C::NC);
      const float *src = A + static_cast<int64_t>(m0 + row) * g.lda + k0 + 4 * c;
      __builtin_amdgcn_global_load_lds((glob_void_t *)src, (lds_void_t *)(ia + j * 1024), 16,
                                       0, 0);
    }
#pragma unroll
    for (int i = 0; i < C::kInstrB; i++) {
      const int j = wid * C::kInstrB + i;
      const int byte = j * 1024 + lane * 16;
      const int kr = byte / C::RBB, pcn = (byte % C::RBB) / 16;
      const int cn = pcn ^ bswz<C>(kr);
      const float *src = B + static_cast<int64_t>(k0 + kr) * g.ldb + n0 + 4 * cn;
      __builtin_amdgcn_global_load_lds((glob_void_t *)src, (lds_void_t *)(ib + j * 1024), 16,
                                       0, 0);
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int r = 0; r < 4; r++) acc[i][j][r] = 0.f;

  const int nk = g.k / BK;
  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * BK);
    const uint8_t *ia = s316_lds + cur * C::kStage;
    const float *ib = reinterpret_cast<const float *>(ia + C::kImgA);
#pragma unroll
    for (int gk = 0; gk < BK / 16; gk++) {
      float4 fa[TM];
      float fb[TN][4];
#pragma unroll
      for (int x = 0; x < TM; x++) {
        const int r = arow + 16 * x;
        fa[x] = *reinterpret_cast<const float4 *>(ia + r * C::RBA +
                                                  swz3<C>(r, 4 * gk + q) * 16);
      }
#pragma unroll
      for (int sidx = 0; sidx < 4; sidx++) {
        const int kr = 16 * gk + 4 * q + sidx;
#pragma unroll
        for (int y = 0; y < TN; y++) {
          const int col = bcol + 16 * y;
          fb[y][sidx] = ib[kr * C::BN + 4 * ((col >> 2) ^ bswz<C>(kr)) + (col & 3)];
        }
      }
#pragma unroll
      for (int sidx = 0; sidx < 4; sidx++)
#pragma unroll
        for (int x = 0; x < TM; x++)
#pragma unroll
          for (int y = 0; y < TN; y++)
            acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(fa[x], sidx), fb[y][sidx],
                                                             acc[x][y], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  const bool use_beta = g.beta != 0.f;
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = n0 + bcol + 16 * y;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = m0 + arow - l16 + 16 * x + 4 * q + r;
        float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
        float v = g.alpha * acc[x][y][r];
        if (use_beta) v += g.beta * *pc;
        *pc = v;
      }
    }
}

template <class C>
bool launch_cfg3x16(const GemmArgs &g, int ta, int tb, bool vec, int batch, hipStream_t s) {
  if (ta || tb || !vec || g.m % C::BM || g.n % C::BN || g.k % C::BK || g.k == 0) return false;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&sgemm3x16_kernel<C>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, C::kLdsBytes);
  const unsigned tiles = static_cast<unsigned>((g.m / C::BM) * (g.n / C::BN));
  hipLaunchKernelGGL(sgemm3x16_kernel<C>, dim3(tiles, 1, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), C::kLdsBytes, s, g);
  return true;
}

// Generation 4: generation 3 (LDS-DMA, 16x16x4 MFMA) with a THREE-stage LDS
// ring so the DMA of tile t+2 stays in flight across the barrier of tile t:
// at the top of tile t each wave waits only for its own DMA of tile t
// (counted vmcnt, tile t+1 left outstanding), a raw s_barrier (no vmcnt(0)
// drain) makes all waves' copies of tile t visible and frees the buffer read
// in tile t-1, then tile t+2's DMA is issued into it and tile t is computed
// (cdna_hip_programming.md "Pipelining across barriers").  BK = 16: one
// 16-k group per tile; A chunk swizzle for 4-chunk rows read by 16x16
// fragments: c ^ 3 * ((row >> 3) & 1) (the 16-lane groups of ds_read_b128
// then hit 16 distinct bank groups).
template <int BM_, int BN_, int WM_, int WN_, bool ASM_ = true, int BK_ = 16>
struct Cfg4 {
  static constexpr int BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_;
  static constexpr int NC = BK / 4;  // 16-byte chunks per A row (4 or 8)
  static_assert(BK == 16 || BK == 32, "BK");
  // fragment reads as inline asm (invisible to the wait-insertion pass); the
  // 1024-thread configuration keeps compiler-visible reads: with asm reads it
  // exceeded its 128-VGPR budget
  static constexpr bool ASM = ASM_;
  static constexpr int kThreads = 64 * WM * WN, kWaves = WM * WN;
  static constexpr int RBA = BK * 4, RBB = BN * 4;
  static constexpr int kImgA = BM * RBA, kImgB = BK * RBB;
  static constexpr int kStage = kImgA + kImgB, kStages = 3;
  static constexpr int kLdsBytes = kStages * kStage;
  static constexpr int kInstrA = kImgA / 1024 / kWaves, kInstrB = kImgB / 1024 / kWaves;
  static constexpr int kInstr = kInstrA + kInstrB;  // DMA instructions per wave per tile
  static_assert(kInstrA * 1024 * kWaves == kImgA && kInstrB * 1024 * kWaves == kImgB,
                "tile not divisible into whole DMA instructions per wave");
  static_assert(kInstr >= 1 && kInstr <= 16, "vmcnt immediates below");
};

// A-image chunk swizzle for 16x16 fragment reads (lanes 0-15 of a quarter
// read rows 0-15 at chunk 4g + q): conflict-free ds_read_b128 groups.
//   4-chunk rows (BK 16):  c ^ 3 ((row >> 3) & 1)
//   8-chunk rows (BK 32):  c ^ ((row >> 1) & 7)
template <int NC>
__device__ __forceinline__ int aswz(int row, int c) {
  if constexpr (NC == 4) return c ^ (3 * ((row >> 3) & 1));
  else return c ^ ((row >> 1) & 7);
}
__device__ __forceinline__ int aswz4(int row, int c) { return aswz<4>(row, c); }

// s_waitcnt vmcnt(N) through the builtin, not inline asm: the compiler's
// wait-insertion pass understands the builtin (an asm wait is opaque to it,
// so it would add its own vmcnt(0) for every DMA it still thinks pending).
// gfx9 encoding: vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt[5:4] << 14.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 0xF) | ((N >> 4) << 14));
}

// The three stages are three distinct __shared__ arrays and the k loop is
// unrolled by three, so every ds_read and every DMA names its array at
// compile time: the compiler's wait insertion can then tell that the DMA in
// flight (another array) does not alias the buffer being read and emits no
// vmcnt(0) before the reads (with one array and a runtime stage index it
// drained the fresh DMA before every tile).
template <class C>
struct Gen4 {
  static constexpr int TM = C::BM / C::WM / 16, TN = C::BN / C::WN / 16;

  __device__ static void stage(uint8_t *ia, const GemmArgs &g, const float *A, const float *B,
                               int m0, int n0, int k0, int wid, int lane) {
    uint8_t *ib = ia + C::kImgA;
#pragma unroll
    for (int i = 0; i < C::kInstrA; i++) {
      const int j = wid * C::kInstrA + i;
      const int row = j * (1024 / C::RBA) + lane / C::NC;
      const int c = aswz<C::NC>(row, lane % C::NC);
      const float *src = A + static_cast<int64_t>(m0 + row) * g.lda + k0 + 4 * c;
      __builtin_amdgcn_global_load_lds((glob_void_t *)src, (lds_void_t *)(ia + j * 1024), 16,
                                       0, 0);
    }
#pragma unroll
    for (int i = 0; i < C::kInstrB; i++) {
      const int j = wid * C::kInstrB + i;
      const int byte = j * 1024 + lane * 16;
      const int kr = byte / C::RBB, pcn = (byte % C::RBB) / 16;
      const int cn = pcn ^ (((kr >> 2) & 1) << 2);
      const float *src = B + static_cast<int64_t>(k0 + kr) * g.ldb + n0 + 4 * cn;
      __builtin_amdgcn_global_load_lds((glob_void_t *)src, (lds_void_t *)(ib + j * 1024), 16,
                                       0, 0);
    }
  }

  // Fragment reads are inline asm: the compiler's wait insertion cannot see
  // them, so it adds no vmcnt(0) for the DMA still in flight into the other
  // stages (with builtin reads it drained the fresh DMA before every second
  // tile).  Ordering is explicit instead: the tile's DMA was retired by the
  // counted vmcnt + barrier before this point, the reads are waited for with
  // lgkmcnt(0), and sched_barrier(0) keeps the MFMAs behind that wait
  // (cdna_hip_programming.md §5.4 rule 18).
  __device__ static void compute(const uint8_t *ia, floatx4 (&acc)[TM][TN], int arow,
                                 int bcol, int q) {
#pragma unroll
    for (int gk = 0; gk < C::BK / 16; gk++) group(ia, acc, arow, bcol, q, gk);
  }

  __device__ static void group(const uint8_t *ia, floatx4 (&acc)[TM][TN], int arow,
                               int bcol, int q, int gk) {
    float4 fa[TM];
    float fb[TN][4];
    if constexpr (!C::ASM) {
      const float *ib = reinterpret_cast<const float *>(ia + C::kImgA);
#pragma unroll
      for (int x = 0; x < TM; x++) {
        const int r = arow + 16 * x;
        fa[x] = *reinterpret_cast<const float4 *>(ia + r * C::RBA +
                                                  aswz<C::NC>(r, 4 * gk + q) * 16);
      }
#pragma unroll
      for (int sidx = 0; sidx < 4; sidx++) {
        const int kr = 16 * gk + 4 * q + sidx;
#pragma unroll
        for (int y = 0; y < TN; y++) {
          const int col = bcol + 16 * y;
          fb[y][sidx] = ib[kr * C::BN + 4 * ((col >> 2) ^ (((kr >> 2) & 1) << 2)) + (col & 3)];
        }
      }
    } else {
      // Fragment reads are inline asm: the compiler's wait insertion cannot
      // see them, so it adds no vmcnt(0) for the DMA still in flight into
      // the other stages.  Ordering is explicit instead: the tile's DMA was
      // retired by the counted vmcnt + barrier before this point, the reads
      // are waited for with lgkmcnt(0), and sched_barrier(0) keeps the MFMAs
      // behind that wait (cdna_hip_programming.md §5.4 rule 18).
      const uint32_t la = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ia));
      const uint32_t lb = la + C::kImgA;
#pragma unroll
      for (int x = 0; x < TM; x++) {
        const int r = arow + 16 * x;
        const uint32_t addr = la + r * C::RBA + aswz<C::NC>(r, 4 * gk + q) * 16;
        asm volatile("ds_read_b128 %0, %1" : "=v"(fa[x]) : "v"(addr) : "memory");
      }
#pragma unroll
      for (int sidx = 0; sidx < 4; sidx++) {
        const int kr = 16 * gk + 4 * q + sidx;
#pragma unroll
        for (int y = 0; y < TN; y++) {
          const int col = bcol + 16 * y;
          const uint32_t addr =
              lb + 4 * (kr * C::BN + 4 * ((col >> 2) ^ (((kr >> 2) & 1) << 2)) + (col & 3));
          asm volatile("ds_read_b32 %0, %1" : "=v"(fb[y][sidx]) : "v"(addr) : "memory");
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int sidx = 0; sidx < 4; sidx++)
#pragma unroll
      for (int x = 0; x < TM; x++)
#pragma unroll
        for (int y = 0; y < TN; y++)
          acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x4f32(comp(fa[x], sidx), fb[y][sidx],
                                                           acc[x][y], 0, 0, 0);
  }
};

template <class C>
__global__ __launch_bounds__(C::kThreads) void sgemm4_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) uint8_t st0[C::kStage];
  __shared__ __attribute__((aligned(1024))) uint8_t st1[C::kStage];
  __shared__ __attribute__((aligned(1024))) uint8_t st2[C::kStage];
  using K = Gen4<C>;
  constexpr int TM = K::TM, TN = K::TN;
  const unsigned tiles_n = g.n / C::BN, tiles_m = g.m / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM, n0 = static_cast<int>(tn) * C::BN;
  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *Cp = g.c + blockIdx.z * g.stride_c;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l16 = lane & 15, q = lane >> 4;
  const int arow = wm * (C::BM / C::WM) + l16;
  const int bcol = wn * (C::BN / C::WN) + l16;

  floatx4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int r = 0; r < 4; r++) acc[i][j][r] = 0.f;

  const int nk = g.k / C::BK;
  K::stage(st0, g, A, B, m0, n0, 0, wid, lane);
  if (nk > 1) K::stage(st1, g, A, B, m0, n0, C::BK, wid, lane);
  // tile kt lives in stage kt % 3; its DMA was issued two tiles earlier
#define VS_GEN4_STEP(CUR, NEXT2)                                              \
  if (kt < nk) {                                                              \
    if (kt + 1 < nk) wait_vmcnt<C::kInstr>();                                 \
    else wait_vmcnt<0>();                                                     \
    __builtin_amdgcn_s_barrier();                                             \
    if (kt + 2 < nk) K::stage(NEXT2, g, A, B, m0, n0, (kt + 2) * C::BK, wid, lane); \
    K::compute(CUR, acc, arow, bcol, q);                                      \
  }                                                                           \
  kt++;
  for (int kt = 0; kt < nk;) {
    VS_GEN4_STEP(st0, st2)
    VS_GEN4_STEP(st1, st0)
    VS_GEN4_STEP(st2, st1)
  }
#undef VS_GEN4_STEP

  const bool use_beta = g.beta != 0.f;
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = n0 + bcol + 16 * y;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = m0 + arow - l16 + 16 * x + 4 * q + r;
        float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
        float v = g.alpha * acc[x][y][r];
        if (use_beta) v += g.beta * *pc;
        *pc = v;
      }
    }
}

template <class C>
bool launch_cfg4(const GemmArgs &g, int ta, int tb, bool vec, int batch, hipStream_t s) {
  if (ta || tb || !vec || g.m % C::BM || g.n % C::BN || g.k % C::BK || g.k == 0) return false;
  const unsigned tiles = static_cast<unsigned>((g.m / C::BM) * (g.n / C::BN));
  hipLaunchKernelGGL(sgemm4_kernel<C>, dim3(tiles, 1, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), 0, s, g);
  return true;
}

// Generation 5: generation 4's three-stage LDS-DMA ring with the whole k loop
// software-pipelined by hand.  Gen 4 lost ~10 % of the MFMA cycles at tile
// boundaries: every wave of a block reached the barrier at the same moment,
// then all of them issued their fragment reads and waited for them, and the
// MFMA pipe ran dry in between (SQ_VALU_MFMA_BUSY 0.905 of 4 x SQ_BUSY_CU at
// 4096^3 against hipBLASLt's 0.978, profiles/r1/pmc_v15_summary.md).  Here
// the barrier sits in the MIDDLE of a tile's MFMA stream:
//
//   tile t:  MFMA k-steps 0,1 from registers R[t&1]
//            wait own DMA of tile t+1 (counted vmcnt) ; s_barrier
//            DMA tile t+3 into tile t's stage (free: its reads all retired)
//            MFMA k-steps 2,3 from R[t&1], one fragment read of tile t+1
//            into R[(t+1)&1] issued after each MFMA
//
// so the reads of the next tile overlap the MFMAs of this one and the next
// tile starts with its fragments already in registers.  MFMAs and fragment
// reads are inline asm (volatile asm keeps program order; the compiler only
// allocates registers), so the interleave is exactly as written; the
// hazards the compiler would otherwise cover are handled explicitly
// (s_nop after the VALU zeroing of the accumulators and before the
// epilogue reads them).  Three stages give each DMA two tiles of cover.
// The dynamic LDS size is padded to kLdsBytes so that exactly the intended
// number of blocks shares a CU.
template <int BM_, int BN_, int WM_, int WN_, int LDS_KB_ = 0, bool AGPR_ = false>
struct Cfg5 {
  static constexpr int BM = BM_, BN = BN_, BK = 16, WM = WM_, WN = WN_;
  // accumulators in AGPRs (MFMA srcC/vdst may be AGPRs): frees the 256
  // architectural VGPRs for fragments when a wave owns a 128 x 128 tile
  static constexpr bool AGPR = AGPR_;
  static constexpr int kThreads = 64 * WM * WN, kWaves = WM * WN;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static constexpr int RBA = BK * 4, RBB = BN * 4;
  static constexpr int kImgA = BM * RBA, kImgB = BK * RBB, kStage = kImgA + kImgB;
  static constexpr int kLdsBytes = 3 * kStage > LDS_KB_ * 1024 ? 3 * kStage : LDS_KB_ * 1024;
  static constexpr int kInstrA = kImgA / 1024 / kWaves, kInstrB = kImgB / 1024 / kWaves;
  static constexpr int kInstr = kInstrA + kInstrB;
  static_assert(kInstrA * 1024 * kWaves == kImgA && kInstrB * 1024 * kWaves == kImgB,
                "tile not divisible into whole DMA instructions per wave");
  static_assert(2 * kInstr < 64, "vmcnt immediates");
  static_assert(TM + 4 * TN <= 2 * TM * TN, "fragment reads must fit between the MFMAs");
};

#define VS_MFMA_16X16X4(ACC, A, B) \
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(ACC) : "v"(A), "v"(B))
#define VS_MFMA_16X16X4_AGPR(ACC, A, B) \
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(ACC) : "v"(A), "v"(B))

template <class C>
struct Gen5 {
  static constexpr int TM = C::TM, TN = C::TN;
  static constexpr int kReads = TM + 4 * TN;
  struct Frag {
    float4 a[TM];
    float b[TN][4];
  };

  // fragment read r of a tile: A rows first (ds_read_b128: 4 k of one row),
  // then B (ds_read_b32, one k of one column)
  template <int R>
  __device__ __forceinline__ static void read(Frag &f, uint32_t va, const uint32_t (&vb)[TN]) {
    if constexpr (R < TM) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.a[R]) : "v"(va), "i"(1024 * R)
                   : "memory");
    } else {
      constexpr int y = (R - TM) / 4, s = (R - TM) % 4;
      asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(f.b[y][s]) : "v"(vb[y]),
                   "i"(4 * s * C::BN) : "memory");
    }
  }

  template <int R = 0>
  __device__ __forceinline__ static void read_all(Frag &f, uint32_t va,
                                                  const uint32_t (&vb)[TN]) {
    if constexpr (R < kReads) {
      read<R>(f, va, vb);
      read_all<R + 1>(f, va, vb);
    }
  }

  // MFMAs number I .. (end of k-steps S0, S0+1); when NEXT is set the
  // fragment read I - I0 of the next tile follows MFMA I
  template <int S0, bool NEXT, int I = 0>
  __device__ __forceinline__ static void mfma_half(floatx4 (&acc)[TM][TN], const Frag &f,
                                                   Frag &nf, uint32_t va,
                                                   const uint32_t (&vb)[TN]) {
    if constexpr (I < 2 * TM * TN) {
      constexpr int s = S0 + I / (TM * TN), x = (I / TN) % TM, y = I % TN;
      if constexpr (C::AGPR) VS_MFMA_16X16X4_AGPR(acc[x][y], comp(f.a[x], s), f.b[y][s]);
      else VS_MFMA_16X16X4(acc[x][y], comp(f.a[x], s), f.b[y][s]);
      if constexpr (NEXT && I < kReads) read<I>(nf, va, vb);
      mfma_half<S0, NEXT, I + 1>(acc, f, nf, va, vb);
    }
  }
};

template <class C>
__global__ __launch_bounds__(C::kThreads) void sgemm5_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t smem5[];
  using K = Gen5<C>;
  constexpr int TM = C::TM, TN = C::TN;
  const unsigned tiles_n = g.n / C::BN, tiles_m = g.m / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM, n0 = static_cast<int>(tn) * C::BN;
  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *Cp = g.c + blockIdx.z * g.stride_c;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l16 = lane & 15, q = lane >> 4;
  const int arow = wm * (C::BM / C::WM) + l16;
  const int bcol = wn * (C::BN / C::WN) + l16;

  // fragment byte offsets inside a stage (see Gen4::group for the layouts):
  // A rows 16x apart differ by 1024 B (the swizzle only depends on row bit 3),
  // B k-steps s differ by 4 * BN B; both go in the instruction's offset field
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem5));
  const uint32_t aoff = arow * C::RBA + 16 * aswz4(arow, q);
  uint32_t boff[TN];
#pragma unroll
  for (int y = 0; y < TN; y++) {
    const int col = bcol + 16 * y;
    boff[y] = C::kImgA + 16 * q * C::BN + 4 * (col & 3) + 16 * ((col >> 2) ^ ((q & 1) << 2));
  }
  // DMA sources for k = 0 (same per-lane mapping as Gen4::stage)
  const float *pa[C::kInstrA];
  const float *pb[C::kInstrB];
#pragma unroll
  for (int i = 0; i < C::kInstrA; i++) {
    const int row = (wid * C::kInstrA + i) * (1024 / C::RBA) + lane / 4;
    pa[i] = A + static_cast<int64_t>(m0 + row) * g.lda + 4 * aswz4(row, lane % 4);
  }
#pragma unroll
  for (int i = 0; i < C::kInstrB; i++) {
    const int byte = (wid * C::kInstrB + i) * 1024 + lane * 16;
    const int kr = byte / C::RBB, pcn = (byte % C::RBB) / 16;
    pb[i] = B + static_cast<int64_t>(kr) * g.ldb + n0 + 4 * (pcn ^ (((kr >> 2) & 1) << 2));
  }
  const auto dma = [&](int st, int kt) {
    uint8_t *base = smem5 + st * C::kStage;
#pragma unroll
    for (int i = 0; i < C::kInstrA; i++)
      __builtin_amdgcn_global_load_lds((glob_void_t *)(pa[i] + kt * C::BK),
                                       (lds_void_t *)(base + (wid * C::kInstrA + i) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < C::kInstrB; i++)
      __builtin_amdgcn_global_load_lds(
          (glob_void_t *)(pb[i] + static_cast<int64_t>(kt) * C::BK * g.ldb),
          (lds_void_t *)(base + C::kImgA + (wid * C::kInstrB + i) * 1024), 16, 0, 0);
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      acc[x][y] = floatx4{0.f, 0.f, 0.f, 0.f};
      // materialise before the s_nop below
      if constexpr (C::AGPR) asm volatile("" : "+a"(acc[x][y]));
      else asm volatile("" : "+v"(acc[x][y]));
    }
  asm volatile("s_nop 7" ::: "memory");  // VALU write -> MFMA srcC read

  const int nk = g.k / C::BK;
  dma(0, 0);
  if (nk > 1) dma(1, 1);
  if (nk > 2) dma(2, 2);
  if (nk > 2) wait_vmcnt<2 * C::kInstr>();
  else if (nk > 1) wait_vmcnt<C::kInstr>();
  else wait_vmcnt<0>();
  __builtin_amdgcn_s_barrier();

  typename K::Frag f0, f1;
  uint32_t vb[TN];
#pragma unroll
  for (int y = 0; y < TN; y++) vb[y] = lds0 + boff[y];
  K::read_all(f0, lds0 + aoff, vb);

  // tile kt: stage kt % 3, registers f[kt & 1].  The MFMA stream is straight
  // line (no branch around it: with one, the register coalescer split the
  // accumulators and copied them at every tile); the last tile's reads of
  // the "next" tile fetch a stale stage and are never used.
#define VS_GEN5_STEP(CUR, NXT)                                                  \
  {                                                                             \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                          \
    K::template mfma_half<0, false>(acc, CUR, NXT, 0u, vb);                     \
    if (kt + 2 < nk) wait_vmcnt<C::kInstr>();                                   \
    else wait_vmcnt<0>();                                                       \
    __builtin_amdgcn_s_barrier();                                               \
    if (kt + 3 < nk) dma(sc, kt + 3);                                           \
    sc = sc == 2 ? 0 : sc + 1;                                                  \
    const uint32_t sb = lds0 + sc * C::kStage;                                  \
    _Pragma("unroll") for (int y = 0; y < TN; y++) vb[y] = sb + boff[y];        \
    K::template mfma_half<2, true>(acc, CUR, NXT, sb + aoff, vb);               \
    kt++;                                                                       \
  }
  int sc = 0;  // stage of tile kt
  for (int kt = 0; kt < nk;) {
    VS_GEN5_STEP(f0, f1)
    if (kt < nk) VS_GEN5_STEP(f1, f0)
  }
#undef VS_GEN5_STEP

  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA -> VALU read
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      if constexpr (C::AGPR) asm volatile("" : "+a"(acc[x][y]));
      else asm volatile("" : "+v"(acc[x][y]));
    }
  const bool use_beta = g.beta != 0.f;
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = n0 + bcol + 16 * y;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = m0 + arow - l16 + 16 * x + 4 * q + r;
        float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
        float v = g.alpha * acc[x][y][r];
        if (use_beta) v += g.beta * *pc;
        *pc = v;
      }
    }
}

template <class C>
bool launch_cfg5(const GemmArgs &g, int ta, int tb, bool vec, int batch, hipStream_t s) {
  if (ta || tb || !vec || g.m % C::BM || g.n % C::BN || g.k % C::BK || g.k == 0) return false;
  (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&sgemm5_kernel<C>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, C::kLdsBytes);
  const unsigned tiles = static_cast<unsigned>((g.m / C::BM) * (g.n / C::BN));
  hipLaunchKernelGGL(sgemm5_kernel<C>, dim3(tiles, 1, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), C::kLdsBytes, s, g);
  return true;
}

using Cfg5A = Cfg5<128, 128, 2, 2, 56>;  // 4 waves of 64 x 64; LDS padded: 2 blocks / CU
using Cfg5B = Cfg5<256, 128, 2, 2, 56>;  // 4 waves of 128 x 64 (128 accumulator VGPRs)
using Cfg5C = Cfg5<128, 128, 2, 2>;      // 48 KiB: up to 3 blocks / CU
using Cfg5D = Cfg5<256, 256, 2, 2, 0, true>;    // 4 waves of 128 x 128, AGPR accumulators
using Cfg5E = Cfg5<256, 128, 2, 2, 56, true>;   // Cfg5B with AGPR accumulators

using Cfg4A = Cfg4<128, 128, 2, 2, false>;  // 48 KiB LDS (3 stages), 4 waves of 64 x 64
using Cfg4B = Cfg4<256, 128, 4, 2>;   // 72 KiB LDS, 8 waves of 64 x 64
using Cfg4C = Cfg4<256, 256, 4, 4, false>;  // 96 KiB LDS, 16 waves of 64 x 64
using Cfg4E = Cfg4<128, 128, 2, 2, true, 32>;   // 96 KiB LDS: 1 block / CU, 1 wave / SIMD
using Cfg4F = Cfg4<128, 128, 2, 2, false, 32>;
using Cfg4G = Cfg4<256, 128, 4, 2, true, 32>;   // 144 KiB LDS

using Cfg3A = Cfg3<256, 128, 32, 4, 2>;   // 96 KiB LDS, 8 waves of 64 x 64
using Cfg3B = Cfg3<128, 128, 32, 2, 2>;   // 64 KiB LDS, 2 blocks / CU
using Cfg3C = Cfg3<256, 256, 16, 4, 2>;   // 64 KiB LDS, 8 waves of 64 x 128

using Cfg2A = Cfg2<128, 128, 32, 2, 2, 1, 1>;
using Cfg2B = Cfg2<256, 128, 32, 4, 2, 1, 1>;
using Cfg2C = Cfg2<128, 256, 32, 2, 4, 1, 1>;

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
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return sgemm_impl(variant, ta, tb, m, n, k, alpha, a + b0 * sa, lda, sa, b + b0 * sb,
                        ldb, sb, beta, c + b0 * sc, ldc, sc, nb, s);
    });
  GemmArgs g{m, n, k, alpha, beta, a, lda, sa, b, ldb, sb, c, ldc, sc};
  const auto al = [](const void *p) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  };
  const bool vec = al(a) && al(b) && lda % 4 == 0 && ldb % 4 == 0 &&
                   (batch == 1 || (sa % 4 == 0 && sb % 4 == 0));
  if (variant < 0) variant = default_variant();
  if (variant < 0) {
    // Largest tile that still gives every CU work (A/B on MI355X,
    // profiles/r1/sgemm_variants.md, sgemm_gen5_ab_v2.log): the LDS-DMA
    // kernels when the shape is NN and whole tiles (gen 5 256x256 from 256
    // tiles, else gen 5 128x128),
    // otherwise 256x128 (gen 1) / 128x128 (gen 2) / 64x64 register-staged.
    const long t128 = static_cast<long>((m + 127) / 128) * ((n + 127) / 128) * batch;
    const long t256 = static_cast<long>((m + 255) / 256) * ((n + 127) / 128) * batch;
    const long t256sq = static_cast<long>((m + 255) / 256) * ((n + 255) / 256) * batch;
    if (t256sq >= 256) variant = 22;       // gen 5 256x256; falls back to 3 unless NN whole tiles
    else if (t128 >= 256) variant = 21;    // gen 5 128x128; falls back to 5
    else if (t256 >= 512) variant = 3;
    else variant = 0;
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
    case 8:
      if (!launch_cfg3<Cfg3A>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 9:
      if (!launch_cfg3<Cfg3B>(g, ta, tb, vec, batch, s)) launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s);
      break;
    case 10:
      if (!launch_cfg3<Cfg3C>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 11:
      if (!launch_cfg3x16<Cfg3A>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 12:
      if (!launch_cfg3x16<Cfg3B>(g, ta, tb, vec, batch, s)) launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s);
      break;
    case 13:
      if (!launch_cfg4<Cfg4A>(g, ta, tb, vec, batch, s)) launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s);
      break;
    case 14:
      if (!launch_cfg4<Cfg4B>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 15:
      if (!launch_cfg4<Cfg4C>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 16:
      if (!launch_cfg4<Cfg4E>(g, ta, tb, vec, batch, s)) launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s);
      break;
    case 17:
      if (!launch_cfg4<Cfg4F>(g, ta, tb, vec, batch, s)) launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s);
      break;
    case 18:
      if (!launch_cfg4<Cfg4G>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 19:
      if (!launch_cfg5<Cfg5A>(g, ta, tb, vec, batch, s)) launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s);
      break;
    case 20:
      if (!launch_cfg5<Cfg5B>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 21:
      if (!launch_cfg5<Cfg5C>(g, ta, tb, vec, batch, s)) launch_cfg2<Cfg2A>(g, ta, tb, vec, batch, s);
      break;
    case 22:
      if (!launch_cfg5<Cfg5D>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;
    case 23:
      if (!launch_cfg5<Cfg5E>(g, ta, tb, vec, batch, s)) launch_cfg<CfgC>(g, ta, tb, vec, batch, s);
      break;

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

// Tuning entry point: run one explicit tile variant (0..15, include/simd/gpu.h).
vs_status vs_sgemm_variant(int variant, int ta, int tb, int m, int n, int k,
                           float alpha, const float *a, int64_t lda,
                           const float *b, int64_t ldb, float beta, float *c,
                           int64_t ldc, vs_stream_t stream) {
  return vs::sgemm_impl(variant, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0,
                        beta, c, ldc, 0, 1, static_cast<hipStream_t>(stream));
}

}  // extern "C"
