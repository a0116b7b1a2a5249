// Exact-fp32 SGEMM on the CDNA4 matrix cores.
//
// gfx950 has no TF32/xf32 path, but it does have an f32-in / f32-accumulate
// MFMA (v_mfma_f32_16x16x4_f32, 64 FLOP/clk/SIMD, bit-exact k-ordered fmaf
// chain) that runs at the full fp32 vector rate (cdna_hip_programming.md §3
// 'FP32-input MFMA').  Two kernel generations remain (earlier register-staged
// and two-stage generations are in git history, profiles/r1/sgemm_variants.md):
//   * gen 5 (sgemm5_kernel): NN, whole 256 x 256 tiles -- a three-stage
//     LDS-DMA ring, hand-pipelined so the barrier sits mid-tile and the next
//     tile's fragment reads interleave with this tile's MFMAs; the default
//     runs 8 waves (2 x 4, two per SIMD, 128 x 64 per wave) so one wave's
//     barrier and LDS waits are covered by the other's MFMAs;
//   * gen 6 (sgemm6_kernel): the same pipeline for every transpose, ragged
//     M / N / K and any alignment, with 256 x 256, 128 x 128 and 64 x 64
//     tiles and split-K for shapes with few output tiles.
// Block ids are remapped so that neighbouring tiles share an XCD's L2 (T1);
// blockIdx.z walks the batch of strided-batched calls.
//
// Reference counterpart: src/matrix.c:200-252 (AVX dot-product GEMM with a
// stack-copied B column, no blocking) and :53-80 (scalar).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "csrc/kernels/device.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glob_void_t;

struct GemmArgs {
  int m, n, k;
  float alpha, beta;
  const float *a;
  int64_t lda, stride_a;
  const float *b;
  int64_t ldb, stride_b;
  float *c;
  int64_t ldc, stride_c;
  // split-K (gen 6): grid.y slices of kchunk k each write partial tiles to
  // c + slice * split_stride (then sgemm_splitk_reduce); kchunk 0 = no split
  int kchunk;
  int64_t split_stride;
};

__device__ __forceinline__ float comp(const float4 &v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}

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
      __builtin_amdgcn_global_load_lds((glob_void_t *)const_cast<float *>(pa[i] + kt * C::BK),
                                       (lds_void_t *)(base + (wid * C::kInstrA + i) * 1024),
                                       16, 0, 0);
#pragma unroll
    for (int i = 0; i < C::kInstrB; i++)
      __builtin_amdgcn_global_load_lds(
          (glob_void_t *)const_cast<float *>(pb[i] + static_cast<int64_t>(kt) * C::BK * g.ldb),
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
  // once per instantiation (a runtime call per launch shows in host-API timings)
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(&sgemm5_kernel<C>),
      hipFuncAttributeMaxDynamicSharedMemorySize, C::kLdsBytes);
  (void)attr;
  const unsigned tiles = static_cast<unsigned>((g.m / C::BM) * (g.n / C::BN));
  hipLaunchKernelGGL(sgemm5_kernel<C>, dim3(tiles, 1, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), C::kLdsBytes, s, g);
  return true;
}

// Generation 6: generation 5's pipeline for every operand layout and shape.
//
// Each operand tile is one of two LDS images, chosen by where K is contiguous:
//   * k-rows  [rows][16] (A as stored for NN/NT, B for NT/TT): one
//     ds_read_b128 per 16-row fragment gives 4 k-steps (the A image of gen 5);
//   * k-major [16][cols] (A for TN/TT, B for NN/TN): one ds_read_b32 per
//     fragment and k-step (the B image of gen 5).
// NT, the reference's matrix_multiply_transposed (src/matrix.c:228-252), is
// the cheapest form: both images are k-rows, so a tile takes TM + TN LDS
// reads instead of TM + 4 TN.
// Both images are filled by buffer-descriptor LDS-DMA (buffer_load ... lds).
// A lane whose source lies past M / N / K gets an out-of-range offset: the
// descriptor's range check returns zeros, so ragged edges need no separate
// path -- zero rows / k slices add nothing, and the epilogue stores only the
// in-range part of the tile.  DMA = 16: 16 bytes per lane (the contiguous
// dimension of both operands a multiple of 4, 16-byte aligned rows);
// DMA = 4: one float per lane for any alignment.
// Rows past the tile base are addressed relative to a per-block descriptor
// base (A + m0 lda, ...), so offsets stay below 2^31 for any matrix whose
// tile-row span fits (checked on the host).
template <int BM_, int BN_, int WM_, int WN_, bool TA_, bool TB_, int DMA_, bool AGPR_,
          int LDS_KB_ = 0, int G_ = 1>
struct Cfg6 {
  static constexpr int BM = BM_, BN = BN_, BK = 16, WM = WM_, WN = WN_;
  // barrier cadence: G = 1, a three-stage ring and a barrier every k tile;
  // G = 2, 4, a ring of 2G stages and a barrier every G tiles (the DMAs of
  // the next G tiles issued behind it)
  static constexpr int G = G_, STAGES = G_ == 1 ? 3 : 2 * G_;
  static_assert(G == 1 || G == 2 || G == 4, "barrier cadence");
  static constexpr bool TA = TA_, TB = TB_, AGPR = AGPR_;
  static constexpr bool AROWS = !TA, BROWS = TB;  // k-rows images
  static constexpr int DMA = DMA_;
  static constexpr int kThreads = 64 * WM * WN, kWaves = WM * WN;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static constexpr int kImgA = BM * 64, kImgB = BN * 64, kStage = kImgA + kImgB;
  static constexpr int kLdsBytes =
      STAGES * kStage > LDS_KB_ * 1024 ? STAGES * kStage : LDS_KB_ * 1024;
  static constexpr int kInstrBytes = 64 * DMA;  // bytes one wave instruction moves
  static constexpr int kInstrA = kImgA / kInstrBytes / kWaves;
  static constexpr int kInstrB = kImgB / kInstrBytes / kWaves;
  static constexpr int kInstr = kInstrA + kInstrB;
  static_assert(kInstrA * kInstrBytes * kWaves == kImgA &&
                    kInstrB * kInstrBytes * kWaves == kImgB,
                "tile not divisible into whole DMA instructions per wave");
  static_assert((STAGES - 1) * kInstr < 64, "vmcnt immediates");
  static constexpr int kReadsA = AROWS ? TM : 4 * TM, kReadsB = BROWS ? TN : 4 * TN;
};

constexpr uint32_t kDmaOut = 0x80000000u;  // an offset past every descriptor's range

// buffer_load_dword{,x4} ... lds of SZ bytes per lane.  The builtin's size
// operand is validated against the compiling target, and the host pass
// (x86) rejects 16 -- which silently dropped the host stubs of every
// 16-byte instantiation -- so the call is compiled for the device only.
template <int SZ>
__device__ __forceinline__ void buffer_dma(__amdgpu_buffer_rsrc_t r, lds_void_t *dst,
                                           uint32_t voff) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (SZ == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, 0, 0, 0);
  else __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 4, voff, 0, 0, 0);
#endif
}

template <class C>
struct Gen6 {
  static constexpr int TM = C::TM, TN = C::TN;
  static constexpr int kReads = C::kReadsA + C::kReadsB;
  struct Frag {
    float4 a4[C::AROWS ? TM : 1];
    float a1[C::AROWS ? 1 : TM][4];
    float4 b4[C::BROWS ? TN : 1];
    float b1[C::BROWS ? 1 : TN][4];
  };
  // LDS byte offsets inside a stage of the fragment reads of lane group q
  // (fragment row / column l16 + 16 x): k-rows images put row r at 64 r
  // with the gen 4 chunk swizzle (16 rows apart = 1024 B: the swizzle only
  // depends on row bit 3); k-major images put k-row kr at kr * 4 cols with
  // the gen 4 column-chunk swizzle by bit 2 of kr, k-step s at + 4 s cols.
  // In a k-major image, fragments x and x + 2 are 128 B apart, but x and
  // x + 1 are not 64 B apart (the swizzle flips the chunk bit that x's
  // parity sets), so odd fragments get their own base: [0] even, [1] odd.
  struct Offs {
    uint32_t a[2], b[2];
  };
  __device__ __forceinline__ static uint32_t kmajor(int col, int q, int ncols) {
    return 16 * q * ncols + 4 * (col & 3) + 16 * ((col >> 2) ^ ((q & 1) << 2));
  }
  __device__ __forceinline__ static Offs offsets(int arow, int bcol, int q) {
    Offs o;
    if constexpr (C::AROWS) o.a[0] = o.a[1] = arow * 64 + 16 * aswz4(arow, q);
    else {
      o.a[0] = kmajor(arow, q, C::BM);
      o.a[1] = kmajor(arow + 16, q, C::BM);
    }
    if constexpr (C::BROWS) o.b[0] = o.b[1] = C::kImgA + bcol * 64 + 16 * aswz4(bcol, q);
    else {
      o.b[0] = C::kImgA + kmajor(bcol, q, C::BN);
      o.b[1] = C::kImgA + kmajor(bcol + 16, q, C::BN);
    }
    return o;
  }
  struct Addr {  // one stage's fragment base addresses
    uint32_t a[2], b[2];
  };
  __device__ __forceinline__ static Addr at(uint32_t stage, const Offs &o) {
    return Addr{{stage + o.a[0], stage + o.a[1]}, {stage + o.b[0], stage + o.b[1]}};
  }

  // Fragment read r of a tile (A first, then B).
  template <int R>
  __device__ __forceinline__ static void read(Frag &f, const Addr &ad) {
    if constexpr (R < C::kReadsA) {
      if constexpr (C::AROWS) {
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.a4[R]) : "v"(ad.a[0]),
                     "i"(1024 * R) : "memory");
      } else {
        constexpr int x = R / 4, st = R % 4;
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(f.a1[x][st]) : "v"(ad.a[x & 1]),
                     "i"(64 * (x & ~1) + 4 * st * C::BM) : "memory");
      }
    } else {
      constexpr int r = R - C::kReadsA;
      if constexpr (C::BROWS) {
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f.b4[r]) : "v"(ad.b[0]),
                     "i"(1024 * r) : "memory");
      } else {
        constexpr int y = r / 4, st = r % 4;
        asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(f.b1[y][st]) : "v"(ad.b[y & 1]),
                     "i"(64 * (y & ~1) + 4 * st * C::BN) : "memory");
      }
    }
  }
  template <int R = 0>
  __device__ __forceinline__ static void read_all(Frag &f, const Addr &ad) {
    if constexpr (R < kReads) {
      read<R>(f, ad);
      read_all<R + 1>(f, ad);
    }
  }
  __device__ __forceinline__ static float opa(const Frag &f, int x, int s) {
    if constexpr (C::AROWS) return comp(f.a4[x], s);
    else return f.a1[x][s];
  }
  __device__ __forceinline__ static float opb(const Frag &f, int y, int s) {
    if constexpr (C::BROWS) return comp(f.b4[y], s);
    else return f.b1[y][s];
  }
  // MFMAs of k-steps S0, S0 + 1; with NEXT, fragment read I of the next tile
  // follows MFMA I, and reads left over after the last MFMA follow it
  template <int S0, bool NEXT, int I = 0>
  __device__ __forceinline__ static void mfma_half(floatx4 (&acc)[TM][TN], const Frag &f,
                                                   Frag &nf, const Addr &ad) {
    if constexpr (I < 2 * TM * TN) {
      constexpr int s = S0 + I / (TM * TN), x = (I / TN) % TM, y = I % TN;
      if constexpr (C::AGPR) VS_MFMA_16X16X4_AGPR(acc[x][y], opa(f, x, s), opb(f, y, s));
      else VS_MFMA_16X16X4(acc[x][y], opa(f, x, s), opb(f, y, s));
      if constexpr (NEXT && I < kReads) read<I>(nf, ad);
      mfma_half<S0, NEXT, I + 1>(acc, f, nf, ad);
    } else if constexpr (NEXT && I < kReads) {
      read<I>(nf, ad);
      mfma_half<S0, NEXT, I + 1>(acc, f, nf, ad);
    }
  }

  // DMA source of wave instruction i (of this wave) for one operand image:
  // byte offset relative to the operand's block base at k0 = 0, the per-tile
  // k stride of that offset, and the row / column and k of the lane.
  struct Src {
    uint32_t off;  // bytes at k0 = 0
    int mn;        // row (k-rows image) or column (k-major image) within the tile
    int kk;        // k within the tile
  };
  template <bool ROWS, int NMN>
  __device__ __forceinline__ static Src src(int J, int lane, int64_t ld) {
    Src r;
    const int byte = J * C::kInstrBytes + lane * C::DMA;
    if constexpr (ROWS) {  // [NMN][16] floats, 64-byte rows, chunk swizzle
      const int row = byte / 64, p = (byte % 64) / 16, w = (byte % 16) / 4;
      const int k = 4 * aswz4(row, p) + w;
      r.mn = row;
      r.kk = k;
      r.off = static_cast<uint32_t>((row * ld + k) * 4);
    } else {  // [16][NMN] floats, column chunk swizzle by k-row bit 2
      const int kr = byte / (4 * NMN), pd = (byte % (4 * NMN)) / 4;
      const int col = 4 * ((pd / 4) ^ (((kr >> 2) & 1) << 2)) + pd % 4;
      r.mn = col;
      r.kk = kr;
      r.off = static_cast<uint32_t>((kr * ld + col) * 4);
    }
    return r;
  }
};

template <class C>
__global__ __launch_bounds__(C::kThreads) void sgemm6_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t smem6[];
  using K = Gen6<C>;
  constexpr int TM = C::TM, TN = C::TN;
  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN, tiles_m = (g.m + C::BM - 1) / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM, n0 = static_cast<int>(tn) * C::BN;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int l16 = lane & 15, q = lane >> 4;
  const int arow = wm * (C::BM / C::WM) + l16;
  const int bcol = wn * (C::BN / C::WN) + l16;

  // per-block descriptors: A rows from m0 (k-rows) or A columns from m0
  // (k-major), B likewise from n0; num_records covers everything, the range
  // check only ever sees kDmaOut
  // split-K slice: k range [kb, kb + kn), partial tile to its own slab
  const int kb = g.kchunk ? static_cast<int>(blockIdx.y) * g.kchunk : 0;
  const int kn = g.kchunk ? min(g.kchunk, g.k - kb) : g.k;
  const float *Ab = g.a + blockIdx.z * g.stride_a + (C::TA ? m0 + kb * g.lda : m0 * g.lda + kb);
  const float *Bb = g.b + blockIdx.z * g.stride_b + (C::TB ? n0 * g.ldb + kb : n0 + kb * g.ldb);
  float *Cp = g.c + blockIdx.z * g.stride_c + blockIdx.y * g.split_stride;
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Ab), 0, 0x7fffffff,
                                                    0x00020000);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Bb), 0, 0x7fffffff,
                                                    0x00020000);
  // DMA lanes: k-rows images advance 16 floats per tile, k-major images
  // 16 rows of ld floats
  typename K::Src sa[C::kInstrA], sb[C::kInstrB];
  bool va[C::kInstrA], vb[C::kInstrB];
#pragma unroll
  for (int i = 0; i < C::kInstrA; i++) {
    sa[i] = K::template src<C::AROWS, C::BM>(wid * C::kInstrA + i, lane, g.lda);
    va[i] = m0 + sa[i].mn < g.m;
  }
#pragma unroll
  for (int i = 0; i < C::kInstrB; i++) {
    sb[i] = K::template src<C::BROWS, C::BN>(wid * C::kInstrB + i, lane, g.ldb);
    vb[i] = n0 + sb[i].mn < g.n;
  }
  const uint32_t stride_a = C::AROWS ? 64u : static_cast<uint32_t>(64 * g.lda);
  const uint32_t stride_b = C::BROWS ? 64u : static_cast<uint32_t>(64 * g.ldb);
  const auto dma = [&](int st, int kt) {
    uint8_t *base = smem6 + st * C::kStage;
    const int k0 = kt * C::BK;
#pragma unroll
    for (int i = 0; i < C::kInstrA; i++) {
      const uint32_t o = va[i] && k0 + sa[i].kk < kn ? sa[i].off + kt * stride_a : kDmaOut;
      buffer_dma<C::DMA>(ra, (lds_void_t *)(base + (wid * C::kInstrA + i) * C::kInstrBytes), o);
    }
#pragma unroll
    for (int i = 0; i < C::kInstrB; i++) {
      const uint32_t o = vb[i] && k0 + sb[i].kk < kn ? sb[i].off + kt * stride_b : kDmaOut;
      buffer_dma<C::DMA>(rb, (lds_void_t *)(base + C::kImgA + (wid * C::kInstrB + i) * C::kInstrBytes),
                         o);
    }
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      acc[x][y] = floatx4{0.f, 0.f, 0.f, 0.f};
      if constexpr (C::AGPR) asm volatile("" : "+a"(acc[x][y]));
      else asm volatile("" : "+v"(acc[x][y]));
    }
  asm volatile("s_nop 7" ::: "memory");  // VALU write -> MFMA srcC read

  const int nk = (kn + C::BK - 1) / C::BK;
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem6));
  const auto off = K::offsets(arow, bcol, q);
  typename K::Frag f0, f1;
  if constexpr (C::G == 1) {
    dma(0, 0);
    if (nk > 1) dma(1, 1);
    if (nk > 2) dma(2, 2);
    if (nk > 2) wait_vmcnt<2 * C::kInstr>();
    else if (nk > 1) wait_vmcnt<C::kInstr>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    K::read_all(f0, K::at(lds0, off));

    // tile kt: stage kt % 3, registers f[kt & 1] (see sgemm5_kernel)
#define VS_GEN6_STEP(CUR, NXT)                                                  \
  {                                                                             \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                          \
    K::template mfma_half<0, false>(acc, CUR, NXT, K::at(0u, off));             \
    if (kt + 2 < nk) wait_vmcnt<C::kInstr>();                                   \
    else wait_vmcnt<0>();                                                       \
    __builtin_amdgcn_s_barrier();                                               \
    if (kt + 3 < nk) dma(sc, kt + 3);                                           \
    sc = sc == 2 ? 0 : sc + 1;                                                  \
    const uint32_t sbase = lds0 + sc * C::kStage;                               \
    K::template mfma_half<2, true>(acc, CUR, NXT, K::at(sbase, off));           \
    kt++;                                                                       \
  }
    int sc = 0;
    for (int kt = 0; kt < nk;) {
      VS_GEN6_STEP(f0, f1)
      if (kt < nk) VS_GEN6_STEP(f1, f0)
    }
  } else {
    // ring of S = 2G stages, stage of tile kt = kt % S.  Prologue: tiles
    // 0..G.  At tiles kt = 0 mod G: wait for this wave's DMAs (tiles
    // kt+1..kt+G, issued one barrier ago), barrier, then refill the stages
    // of tiles kt-G+1..kt -- every wave has read them (tile kt's reads were
    // waited at its start) -- with tiles kt+G+1..kt+2G.  Between barriers
    // the waves read tiles kt+1..kt+G, all covered by this barrier.
    constexpr int G = C::G, S = C::STAGES;
#pragma unroll
    for (int j = 0; j <= G; j++)
      if (j < nk) dma(j, j);
    if (nk > G) wait_vmcnt<G * C::kInstr>();
    else wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    K::read_all(f0, K::at(lds0, off));
#define VS_GEN6_STEPG(CUR, NXT)                                                 \
  {                                                                             \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                          \
    K::template mfma_half<0, false>(acc, CUR, NXT, K::at(0u, off));             \
    if ((kt & (G - 1)) == 0) {                                                  \
      wait_vmcnt<0>();                                                          \
      __builtin_amdgcn_s_barrier();                                             \
      _Pragma("unroll") for (int j = 1; j <= G; j++) {                          \
        if (kt + G + j < nk) dma((kt + G + j) & (S - 1), kt + G + j);           \
      }                                                                         \
    }                                                                           \
    const uint32_t sbase = lds0 + ((kt + 1) & (S - 1)) * C::kStage;             \
    K::template mfma_half<2, true>(acc, CUR, NXT, K::at(sbase, off));           \
    kt++;                                                                       \
  }
    for (int kt = 0; kt < nk;) {
      VS_GEN6_STEPG(f0, f1)
      if (kt < nk) VS_GEN6_STEPG(f1, f0)
    }
#undef VS_GEN6_STEPG
  }
#undef VS_GEN6_STEP

  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA -> VALU read
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      if constexpr (C::AGPR) asm volatile("" : "+a"(acc[x][y]));
      else asm volatile("" : "+v"(acc[x][y]));
    }
  const bool use_beta = g.beta != 0.f;
  const bool interior = m0 + C::BM <= g.m && n0 + C::BN <= g.n;
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = n0 + bcol + 16 * y;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = m0 + arow - l16 + 16 * x + 4 * q + r;
        if (interior || (row < g.m && col < g.n)) {
          float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
          float v = g.alpha * acc[x][y][r];
          if (use_beta) v += g.beta * *pc;
          *pc = v;
        }
      }
    }
}

// Generation 7: gen 6's images and fragment layouts with the issue stream of
// the steady-state k loop laid out for two waves per SIMD.
//
// PMC on gen 5 / 6 put the MFMA pipe at 0.92-0.93 busy where hipBLASLt's
// kernel reaches 0.98 with the same instruction count.  The idle share sat
// right behind each tile's barrier: every wave ran the same burst there --
// three scalar branches, v_readfirstlane + s_mov m0 pairs (the wave id came
// from threadIdx, which the compiler treats as divergent), 64-bit VALU
// address adds and all of the tile's LDS-DMA pieces back to back (a piece
// holds the issuing wave for ~60 cycles) -- and with both waves of a SIMD in
// lockstep nobody fed the matrix pipe meanwhile.  Here:
//   * the wave id is made uniform once (readfirstlane), DMA voffsets are
//     loop invariant and the k advance travels in the instruction's scalar
//     soffset, so a piece is s_mov m0 + buffer_load ... lds and nothing else;
//   * full tiles run in a branch-free loop (the last tiles, whose DMAs are
//     absent or k-masked, run gen 6's generic step);
//   * the pieces are spread over the MFMA gaps behind the fragment reads;
//   * with 8 waves, waves 4-7 (the SIMD partners of waves 0-3) run half a
//     tile out of phase inside each barrier interval: group X does
//     [reads + DMA + MFMA | MFMA only | barrier], group Y
//     [MFMA only | reads + DMA + MFMA | barrier], so one partner always has
//     bare MFMAs to issue while the other sits in an LDS / DMA issue slot.
//     Every wave still passes the same barriers: b_t, which publishes tile
//     t + 1 and frees tile t's stage, is X's mid-tile barrier of tile t and
//     Y's end-of-tile barrier of tile t - 1 (Y passes b_0 in its prologue and
//     none after its last tile: nk + 1 barriers per wave on either path).
template <class C>
struct Gen7 {
  using K = Gen6<C>;
  static constexpr int TM = C::TM, TN = C::TN, N = 2 * TM * TN;
  // MFMA gap (index within the load half) that takes DMA piece j: spread
  // evenly behind the fragment reads
  static constexpr int slot(int j) {
    if (K::kReads + C::kInstr >= N) return N - 1 - (C::kInstr - 1 - j) % N;
    return K::kReads + (j + 1) * (N - K::kReads) / (C::kInstr + 1);
  }
  template <int I, int J, class D>
  __device__ __forceinline__ static void pieces(const D &d) {
    if constexpr (J < C::kInstr) {
      if constexpr (slot(J) == I) d(std::integral_constant<int, J>{});
      pieces<I, J + 1>(d);
    }
  }
  template <int J, class D>
  __device__ __forceinline__ static void pieces_all(const D &d) {
    if constexpr (J < C::kInstr) {
      d(std::integral_constant<int, J>{});
      pieces_all<J + 1>(d);
    }
  }
  // MFMAs of k-steps S0, S0 + 1; LOAD: fragment read I of the next tile and
  // the DMA pieces of gap I follow MFMA I
  template <int S0, bool LOAD, class D, int I = 0>
  __device__ __forceinline__ static void half(floatx4 (&acc)[TM][TN], const typename K::Frag &f,
                                              typename K::Frag &nf, const typename K::Addr &ad,
                                              const D &d) {
    if constexpr (I < N) {
      constexpr int s = S0 + I / (TM * TN), x = (I / TN) % TM, y = I % TN;
      if constexpr (C::AGPR) VS_MFMA_16X16X4_AGPR(acc[x][y], K::opa(f, x, s), K::opb(f, y, s));
      else VS_MFMA_16X16X4(acc[x][y], K::opa(f, x, s), K::opb(f, y, s));
      if constexpr (LOAD && I < K::kReads) K::template read<I>(nf, ad);
      if constexpr (LOAD) pieces<I, 0>(d);
      half<S0, LOAD, D, I + 1>(acc, f, nf, ad, d);
    } else if constexpr (LOAD && I < K::kReads) {
      K::template read<I>(nf, ad);
      half<S0, LOAD, D, I + 1>(acc, f, nf, ad, d);
    }
  }
};

template <int SZ>
__device__ __forceinline__ void buffer_dma_s(__amdgpu_buffer_rsrc_t r, lds_void_t *dst,
                                             uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (SZ == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
  else __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 4, voff, soff, 0, 0);
#endif
}

// One wave's whole tile; Y selects the wave group's phase (see Gen7).  The
// two groups are separate instantiations called from a uniform branch, each
// with its own accumulators from zeroing to store (accumulators live across
// the branch made the register allocator copy / spill them at the join).
// Every step issues its kInstr DMA pieces: lanes at or past the end of K --
// the ragged part of the last tile, and whole tiles past it -- get the
// out-of-range offset, so they fill their (free) stage with zeros; the
// counted vmcnt is then the same in every step and the k loop has no branch
// but its back edge.
template <class C, bool Y>
__device__ __forceinline__ void sgemm7_run(const GemmArgs &g, uint8_t *smem7, int wid) {
  using K = Gen6<C>;
  using K7 = Gen7<C>;
  static_assert(C::G == 1, "three-stage ring");
  constexpr int TM = C::TM, TN = C::TN;
  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN, tiles_m = (g.m + C::BM - 1) / C::BM;
  const unsigned t = dev::xcd_remap(blockIdx.x, tiles_m * tiles_n);
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM, n0 = static_cast<int>(tn) * C::BN;
  const int lane = threadIdx.x & 63;
  const int wm = wid / C::WN, wn = wid % C::WN;

  const int kb = g.kchunk ? static_cast<int>(blockIdx.y) * g.kchunk : 0;
  const int kn = g.kchunk ? min(g.kchunk, g.k - kb) : g.k;
  const float *Ab = g.a + blockIdx.z * g.stride_a + (C::TA ? m0 + kb * g.lda : m0 * g.lda + kb);
  const float *Bb = g.b + blockIdx.z * g.stride_b + (C::TB ? n0 * g.ldb + kb : n0 + kb * g.ldb);
  float *Cp = g.c + blockIdx.z * g.stride_c + blockIdx.y * g.split_stride;
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Ab), 0, 0x7fffffff,
                                                    0x00020000);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Bb), 0, 0x7fffffff,
                                                    0x00020000);
  // loop-invariant DMA voffsets (row / column mask folded in) and k positions
  uint32_t voa[C::kInstrA], vob[C::kInstrB];
  int kka[C::kInstrA], kkb[C::kInstrB];
#pragma unroll
  for (int i = 0; i < C::kInstrA; i++) {
    const auto sa = K::template src<C::AROWS, C::BM>(wid * C::kInstrA + i, lane, g.lda);
    voa[i] = m0 + sa.mn < g.m ? sa.off : kDmaOut;
    kka[i] = sa.kk;
  }
#pragma unroll
  for (int i = 0; i < C::kInstrB; i++) {
    const auto sb = K::template src<C::BROWS, C::BN>(wid * C::kInstrB + i, lane, g.ldb);
    vob[i] = n0 + sb.mn < g.n ? sb.off : kDmaOut;
    kkb[i] = sb.kk;
  }
  const uint32_t stride_a = C::AROWS ? 64u : static_cast<uint32_t>(64 * g.lda);
  const uint32_t stride_b = C::BROWS ? 64u : static_cast<uint32_t>(64 * g.ldb);
  uint8_t *const wbase_a = smem7 + wid * C::kInstrA * C::kInstrBytes;
  uint8_t *const wbase_b = smem7 + C::kImgA + wid * C::kInstrB * C::kInstrBytes;
  const int nk = (kn + C::BK - 1) / C::BK;
  // DMA piece J of tile kt into stage st
  const auto piece_of = [&](auto jc, int st, int kt) {
    constexpr int J = decltype(jc)::value;
    const int rem = kn - kt * C::BK;        // <= 0 for tiles past the end
    const int ktc = min(kt, nk - 1);        // keeps soffset inside the operand
    if constexpr (J < C::kInstrA) {
      const uint32_t o = kka[J] < rem ? voa[J] : kDmaOut;
      buffer_dma_s<C::DMA>(ra, (lds_void_t *)(wbase_a + st * C::kStage + J * C::kInstrBytes), o,
                           ktc * stride_a);
    } else {
      constexpr int j = J - C::kInstrA;
      const uint32_t o = kkb[j] < rem ? vob[j] : kDmaOut;
      buffer_dma_s<C::DMA>(rb, (lds_void_t *)(wbase_b + st * C::kStage + j * C::kInstrBytes), o,
                           ktc * stride_b);
    }
  };
  const auto dma_all = [&](int st, int kt) {
    K7::template pieces_all<0>([&](auto jc) { piece_of(jc, st, kt); });
  };

  floatx4 acc[TM][TN];
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      acc[x][y] = floatx4{0.f, 0.f, 0.f, 0.f};
      if constexpr (C::AGPR) asm volatile("" : "+a"(acc[x][y]));
      else asm volatile("" : "+v"(acc[x][y]));
    }
  asm volatile("s_nop 7" ::: "memory");  // VALU write -> MFMA srcC read

  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem7));
  typename K::Offs off;
  {
    const int l16 = lane & 15, q = lane >> 4;
    off = K::offsets(wm * (C::BM / C::WM) + l16, wn * (C::BN / C::WN) + l16, q);
  }
  typename K::Frag f0, f1;

  dma_all(0, 0);
  dma_all(1, 1);
  dma_all(2, 2);
  wait_vmcnt<2 * C::kInstr>();
  __builtin_amdgcn_s_barrier();
  K::read_all(f0, K::at(lds0, off));
  if constexpr (Y) {  // b_0: tile 1 published
    wait_vmcnt<C::kInstr>();
    __builtin_amdgcn_s_barrier();
  }

  const auto nodma = [](auto) {};
  int sc = 0;  // stage of tile kt
  // tile kt from registers CUR; reads tile kt + 1 into NXT; DMA of tile kt + 3
#define VS_GEN7_STEP(CUR, NXT)                                                        \
  {                                                                                   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                \
    K7::template half<0, false>(acc, CUR, NXT, K::at(0u, off), nodma);                \
    if constexpr (!Y) {                                                               \
      wait_vmcnt<C::kInstr>();                                                        \
      __builtin_amdgcn_s_barrier();                                                   \
    }                                                                                 \
    const int st = sc, kd = kt + 3;                                                   \
    sc = sc == 2 ? 0 : sc + 1;                                                        \
    K7::template half<2, true>(acc, CUR, NXT, K::at(lds0 + sc * C::kStage, off),      \
                               [&](auto jc) { piece_of(jc, st, kd); });               \
    kt++;                                                                             \
    if constexpr (Y) {                                                                \
      if (kt < nk) {                                                                  \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                            \
        wait_vmcnt<C::kInstr>();                                                      \
        __builtin_amdgcn_s_barrier();                                                 \
      }                                                                               \
    }                                                                                 \
  }
  for (int kt = 0; kt < nk;) {
    VS_GEN7_STEP(f0, f1)
    if (kt < nk) VS_GEN7_STEP(f1, f0)
  }
#undef VS_GEN7_STEP
  // zero-fill DMAs of the tiles past the end may still be in flight: LDS
  // must not be handed to the next block's waves before they land
  wait_vmcnt<0>();

  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");  // MFMA -> VALU read
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      if constexpr (C::AGPR) asm volatile("" : "+a"(acc[x][y]));
      else asm volatile("" : "+v"(acc[x][y]));
    }
  int ln = lane;  // store coordinates recomputed here: no registers held across the loop
  asm volatile("" : "+v"(ln));
  const int l16 = ln & 15, q = ln >> 4;
  const int arow = wm * (C::BM / C::WM) + l16;
  const int bcol = wn * (C::BN / C::WN) + l16;
  const bool use_beta = g.beta != 0.f;
  const bool interior = m0 + C::BM <= g.m && n0 + C::BN <= g.n;
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = n0 + bcol + 16 * y;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = m0 + arow - l16 + 16 * x + 4 * q + r;
        if (interior || (row < g.m && col < g.n)) {
          float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
          float v = g.alpha * acc[x][y][r];
          if (use_beta) v += g.beta * *pc;
          *pc = v;
        }
      }
    }
}

template <class C>
__global__ __launch_bounds__(C::kThreads) void sgemm7_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t smem7[];
  const int wid = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if constexpr (C::kWaves == 8) {
    if (wid >= 4) sgemm7_run<C, true>(g, smem7, wid);
    else sgemm7_run<C, false>(g, smem7, wid);
  } else {
    sgemm7_run<C, false>(g, smem7, wid);
  }
}

// Whether gen 6 can address this call: every DMA offset of a block below
// 2^31 bytes relative to its block base.
template <class C>
bool gen6_fits(const GemmArgs &g) {
  const int64_t ka = C::TA ? static_cast<int64_t>(g.k) * g.lda : static_cast<int64_t>(C::BM) * g.lda;
  const int64_t kb = C::TB ? static_cast<int64_t>(C::BN) * g.ldb : static_cast<int64_t>(g.k) * g.ldb;
  return g.k > 0 && 4 * (ka + 64) < (1LL << 31) && 4 * (kb + 64) < (1LL << 31);
}

template <class C, bool GEN7 = false>
bool launch_cfg6(const GemmArgs &g, int batch, hipStream_t s) {
  if (!gen6_fits<C>(g)) return false;
  void (*kern)(GemmArgs);
  if constexpr (GEN7) kern = &sgemm7_kernel<C>;
  else kern = &sgemm6_kernel<C>;
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(kern),
      hipFuncAttributeMaxDynamicSharedMemorySize, C::kLdsBytes);
  (void)attr;
  const unsigned tiles = static_cast<unsigned>(((g.m + C::BM - 1) / C::BM) *
                                               ((g.n + C::BN - 1) / C::BN));
  const unsigned splits = g.kchunk ? static_cast<unsigned>((g.k + g.kchunk - 1) / g.kchunk) : 1;
  hipLaunchKernelGGL(kern, dim3(tiles, splits, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), C::kLdsBytes, s, g);
  return true;
}

// c[b] = alpha * sum_s w[b][s] + beta * c[b] over m x n (w slabs m x n dense).
__global__ __launch_bounds__(256) void sgemm_splitk_reduce(const float *__restrict__ w,
                                                           int splits, int64_t slab, int m,
                                                           int n, float alpha, float beta,
                                                           float *__restrict__ c, int64_t ldc,
                                                           int64_t stride_c) {
  const int64_t mn = static_cast<int64_t>(m) * n;
  const float *wb = w + blockIdx.y * slab * splits;
  float *cb = c + blockIdx.y * stride_c;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < mn; i += static_cast<int64_t>(gridDim.x) * 256) {
    float acc = 0.f;
    for (int s = 0; s < splits; s++) acc += wb[s * slab + i];
    const int64_t r = i / n, col = i - r * n;
    float *pc = cb + r * ldc + col;
    *pc = beta != 0.f ? alpha * acc + beta * *pc : alpha * acc;
  }
}

// Tile geometry x transposes x DMA width.
template <int BM, int BN, int WM, int WN, int DMA, bool AGPR, int LDS_KB, int G = 1,
          bool GEN7 = false>
bool launch_gen6_t(const GemmArgs &g, int ta, int tb, int batch, hipStream_t s) {
  if (!ta && !tb)
    return launch_cfg6<Cfg6<BM, BN, WM, WN, false, false, DMA, AGPR, LDS_KB, G>, GEN7>(g, batch, s);
  if (!ta && tb)
    return launch_cfg6<Cfg6<BM, BN, WM, WN, false, true, DMA, AGPR, LDS_KB, G>, GEN7>(g, batch, s);
  if (ta && !tb)
    return launch_cfg6<Cfg6<BM, BN, WM, WN, true, false, DMA, AGPR, LDS_KB, G>, GEN7>(g, batch, s);
  return launch_cfg6<Cfg6<BM, BN, WM, WN, true, true, DMA, AGPR, LDS_KB, G>, GEN7>(g, batch, s);
}

// 16-byte DMA needs 16-byte aligned operand rows whose contiguous dimension
// (k for k-rows images, m / n for k-major ones) is a multiple of 4.
bool gen6_dma16(const GemmArgs &g, int ta, int tb, int batch) {
  const auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int ca = ta ? g.m : g.k, cb = tb ? g.k : g.n;
  return al(g.a) && al(g.b) && g.lda % 4 == 0 && g.ldb % 4 == 0 && ca % 4 == 0 &&
         cb % 4 == 0 && (batch == 1 || (g.stride_a % 4 == 0 && g.stride_b % 4 == 0));
}

// tile: 0 = 128 x 128 (4 waves of 64 x 64), 1 = 256 x 256 (4 waves of
// 128 x 128, AGPR accumulators), 2 = 64 x 64 (4 waves of 32 x 32),
// 3 / 4 = 256 x 256 with 8 waves (2 x 4 / 4 x 2, two per SIMD), 5 = 128 x 128
// with 8 waves (2 x 4), 6 = 2 with an eight-stage ring (64 KiB: two blocks
// per CU) and a barrier every four k tiles; 4-byte DMA
// at 128 x 128 / 64 x 64 only (vmcnt range).
bool launch_gen6_tile(const GemmArgs &g, int ta, int tb, int batch, hipStream_t s, int tile) {
  const bool d16 = gen6_dma16(g, ta, tb, batch);
  // gen 7 (16-byte DMA only): 7 = 256 x 256 8 waves, 8 = 128 x 128 8 waves,
  // 9 = 128 x 128 4 waves, 10 = 256 x 256 4 waves
  if (tile == 7 && d16) return launch_gen6_t<256, 256, 2, 4, 16, true, 0, 1, true>(g, ta, tb, batch, s);
  if (tile == 8 && d16) return launch_gen6_t<128, 128, 2, 4, 16, false, 0, 1, true>(g, ta, tb, batch, s);
  if (tile == 9 && d16) return launch_gen6_t<128, 128, 2, 2, 16, false, 0, 1, true>(g, ta, tb, batch, s);
  if (tile == 10 && d16) return launch_gen6_t<256, 256, 2, 2, 16, true, 0, 1, true>(g, ta, tb, batch, s);
  if (tile == 7 || tile == 10) tile = 3;
  if (tile == 8) tile = 5;
  if (tile == 9) tile = 0;
  if (tile == 1 && d16) return launch_gen6_t<256, 256, 2, 2, 16, true, 0>(g, ta, tb, batch, s);
  if (tile == 3 && d16) return launch_gen6_t<256, 256, 2, 4, 16, true, 0>(g, ta, tb, batch, s);
  if (tile == 4 && d16) return launch_gen6_t<256, 256, 4, 2, 16, true, 0>(g, ta, tb, batch, s);
  if (tile == 5) {  // 128 x 128 with 8 waves (2 x 4 of 64 x 32)
    if (d16) return launch_gen6_t<128, 128, 2, 4, 16, false, 0>(g, ta, tb, batch, s);
    return launch_gen6_t<128, 128, 2, 4, 4, false, 0>(g, ta, tb, batch, s);
  }
  if (tile == 6) {  // 64 x 64, 4 waves, barrier every 4 k tiles (2 otherwise)
    if (d16) return launch_gen6_t<64, 64, 2, 2, 16, false, 0, 4>(g, ta, tb, batch, s);
    tile = 2;
  }
  if (tile == 2) {
    if (d16) return launch_gen6_t<64, 64, 2, 2, 16, false, 0>(g, ta, tb, batch, s);
    return launch_gen6_t<64, 64, 2, 2, 4, false, 0>(g, ta, tb, batch, s);
  }
  if (d16) return launch_gen6_t<128, 128, 2, 2, 16, false, 0>(g, ta, tb, batch, s);
  return launch_gen6_t<128, 128, 2, 2, 4, false, 0>(g, ta, tb, batch, s);
}

// Split-K count for `tiles` output tiles: k slices of >= 256 until
// tiles x slices reaches ~2 per CU.
int auto_splits(long tiles, int k) {
  const long want = 2L * device_cu_count();
  int splits = 1;
  while (tiles * splits * 2 <= want && k / (splits * 2) >= 256) splits *= 2;
  return splits;
}

// Gen 6 with split-K when the output tiles cannot fill the chip: k slices
// of >= 256 (a multiple of 16) until tiles x slices reaches ~2 per CU,
// partial tiles to a workspace, one reduction pass applying alpha / beta.
bool launch_gen6(const GemmArgs &g0, int ta, int tb, int batch, hipStream_t s, int tile,
                 int splits = 0) {
  const int bm = (tile == 1 || tile == 3 || tile == 4 || tile == 7 || tile == 10) ? 256
                 : (tile == 2 || tile == 6)                                       ? 64
                                                                                  : 128;
  const long tiles = static_cast<long>((g0.m + bm - 1) / bm) * ((g0.n + bm - 1) / bm) * batch;
  if (splits <= 0) splits = auto_splits(tiles, g0.k);
  if (splits <= 1) {
    GemmArgs g = g0;
    g.kchunk = 0;
    return launch_gen6_tile(g, ta, tb, batch, s, tile);
  }
  GemmArgs g = g0;
  g.kchunk = ((g.k + splits - 1) / splits + 15) / 16 * 16;
  splits = (g.k + g.kchunk - 1) / g.kchunk;
  const int64_t slab = static_cast<int64_t>(g.m) * g.n;
  DeviceBuffer ws;
  if (ws.alloc(sizeof(float) * slab * splits * batch, s) != VS_OK) return false;
  g.c = ws.as<float>();
  g.ldc = g.n;
  g.split_stride = slab;
  g.stride_c = slab * splits;
  g.alpha = 1.f;
  g.beta = 0.f;
  if (!launch_gen6_tile(g, ta, tb, batch, s, tile)) return false;
  const unsigned blocks = static_cast<unsigned>(std::min<int64_t>((slab + 255) / 256, 4096));
  hipLaunchKernelGGL(sgemm_splitk_reduce, dim3(blocks, static_cast<unsigned>(batch)), dim3(256),
                     0, s, ws.as<float>(), splits, slab, g0.m, g0.n, g0.alpha, g0.beta, g0.c,
                     g0.ldc, g0.stride_c);
  return true;
}

using Cfg5D = Cfg5<256, 256, 2, 2, 0, true>;
// 8-wave gen-5 tiles (two waves per SIMD: one wave's barrier / LDS waits
// are filled by the other's MFMAs; 128 accumulator AGPRs per wave)
using Cfg5W24 = Cfg5<256, 256, 2, 4, 0, true>;
using Cfg5W42 = Cfg5<256, 256, 4, 2, 0, true>;  // 4 waves of 128 x 128, AGPR accumulators

__global__ __launch_bounds__(256) void scale_c_kernel(int m, int n, float beta,
                                                      float *__restrict__ c, int64_t ldc,
                                                      int64_t stride_c) {
  const int64_t mn = static_cast<int64_t>(m) * n;
  float *cb = c + blockIdx.y * stride_c;
  for (int64_t i = blockIdx.x * 256LL + threadIdx.x; i < mn;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    const int64_t r = i / n;
    float *p = cb + r * ldc + (i - r * n);
    *p = beta != 0.f ? beta * *p : 0.f;
  }
}

int default_variant() {
  static const int v = [] {
    const char *e = std::getenv("VELES_SGEMM_VARIANT");
    return e && *e ? std::atoi(e) : -1;
  }();
  return v;
}

// Default kernel choice: for each candidate (tile, workgroups per CU,
// relative per-CU throughput), the split-K count launch_gen6 would use and
// the wave-quantisation efficiency of tiles x splits over CUs x slots; the
// best modelled score wins, larger tiles on ties.  Calibrated on MI355X
// (profiles/r2/sgemm_w8_ab.md): 256 x 256 8-wave 1 / CU at 1.0, 128 x 128
// 8-wave 2 / CU at 0.94, 64 x 64 4-wave 4 / CU at 0.90, split-K passes x 0.95.
// When the 64 x 64 blocks (split-K slices included) fit two per CU, the
// eight-stage, barrier-every-four-tiles build (64 KiB LDS, still two per
// CU) runs instead: a lone 4-wave block per SIMD set does only 16 MFMAs per
// wave between barriers at one k tile per barrier (512^3 21.7 -> 22.6,
// 300 x 1000 x 256 NN / NT 17.2 -> 18.1 / 18.5 -> 19.4 TF, 1000^3 flat; with
// more blocks than two per CU it loses 6-9 %, the bigger ring stopping
// blocks from sharing a CU: profiles/r2/session6/sgemm_barrier_cadence.md).
int pick_variant(int m, int n, int k, int batch) {
  const long cus = device_cu_count();
  const auto eff = [&](long work, long slots) {
    const long waves = (work + slots - 1) / slots;
    return static_cast<double>(work) / static_cast<double>(waves * slots);
  };
  const long t256 = static_cast<long>((m + 255) / 256) * ((n + 255) / 256) * batch;
  const long t128 = static_cast<long>((m + 127) / 128) * ((n + 127) / 128) * batch;
  const long t64 = static_cast<long>((m + 63) / 64) * ((n + 63) / 64) * batch;
  const int s128 = auto_splits(t128, k), s64 = auto_splits(t64, k);
  const double a = eff(t256, cus);
  const double b = 0.94 * eff(t128 * s128, 2 * cus) * (s128 > 1 ? 0.95 : 1.0);
  const double c = 0.90 * eff(t64 * s64, 4 * cus) * (s64 > 1 ? 0.95 : 1.0);
  if (a >= b && a >= c) return 6;
  if (b >= c) return s128 > 1 ? 9 : 8;
  return t64 * s64 <= 2 * cus ? 10 : 4;
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
  if (k == 0) {  // no product: C = beta C (C = 0 for beta = 0, NaN included)
    const int64_t mn = static_cast<int64_t>(m) * n;
    hipLaunchKernelGGL(scale_c_kernel, dim3(elementwise_grid(mn, 256), batch), dim3(256), 0, s,
                       m, n, beta, c, ldc, sc);
    VS_HIP(hipGetLastError());
    return VS_OK;
  }
  GemmArgs g{m, n, k, alpha, beta, a, lda, sa, b, ldb, sb, c, ldc, sc, 0, 0};
  if (variant < 0) variant = default_variant();
  if (variant < 0) variant = pick_variant(m, n, k, batch);
  bool ok = false;
#ifdef VS_SGEMM_PROBE
  ok = launch_cfg6<Cfg6<256, 256, 2, VS_SGEMM_PROBE, false, false, 16, true, 0, 1>, true>(g, batch, s);
#else
  switch (variant) {
    case 0: ok = launch_gen6(g, ta, tb, batch, s, 2, 1); break;   // 64 x 64
    case 1: ok = launch_gen6(g, ta, tb, batch, s, 0, 1); break;   // 128 x 128
    case 2: ok = launch_gen6(g, ta, tb, batch, s, 1, 1); break;   // 256 x 256
    case 3:                                                       // gen 5 NN, else 256 x 256
      ok = launch_cfg5<Cfg5D>(g, ta, tb, gen6_dma16(g, ta, tb, batch), batch, s) ||
           launch_gen6(g, ta, tb, batch, s, 1, 1);
      break;
    case 4: ok = launch_gen6(g, ta, tb, batch, s, 2); break;      // 64 x 64, split-K
    case 5: ok = launch_gen6(g, ta, tb, batch, s, 0); break;      // 128 x 128, split-K
    case 6:  // 256 x 256 with 8 waves (2 x 4, two per SIMD): gen 5 NN, else gen 6
      ok = launch_cfg5<Cfg5W24>(g, ta, tb, gen6_dma16(g, ta, tb, batch), batch, s) ||
           launch_gen6(g, ta, tb, batch, s, 3, 1);
      break;
    case 7:  // 256 x 256 with 8 waves (4 x 2): gen 5 NN, else gen 6
      ok = launch_cfg5<Cfg5W42>(g, ta, tb, gen6_dma16(g, ta, tb, batch), batch, s) ||
           launch_gen6(g, ta, tb, batch, s, 4, 1);
      break;
    case 8: ok = launch_gen6(g, ta, tb, batch, s, 5, 1); break;  // 128 x 128, 8 waves
    case 9: ok = launch_gen6(g, ta, tb, batch, s, 5); break;     // same, split-K
    case 10: ok = launch_gen6(g, ta, tb, batch, s, 6); break;     // 4, barrier / 4 k tiles
    case 11: ok = launch_gen6(g, ta, tb, batch, s, 7, 1); break;  // gen 7 256 x 256, 8 waves
    case 12: ok = launch_gen6(g, ta, tb, batch, s, 8, 1); break;  // gen 7 128 x 128, 8 waves
    case 13: ok = launch_gen6(g, ta, tb, batch, s, 9, 1); break;  // gen 7 128 x 128, 4 waves
    case 14: ok = launch_gen6(g, ta, tb, batch, s, 10, 1); break; // gen 7 256 x 256, 4 waves
    default:
      set_error("vs_sgemm: unknown variant %d (0..%d)", variant, VS_SGEMM_VARIANTS - 1);
      return VS_ERR_INVALID;
  }
#endif
  VS_REQUIRE(ok, "vs_sgemm: operand spans beyond 2^31 bytes per tile row (m %d n %d k %d)", m,
             n, k);
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

// Tuning entry point: run one explicit kernel variant (0..VS_SGEMM_VARIANTS-1,
// include/simd/gpu.h).
vs_status vs_sgemm_variant(int variant, int ta, int tb, int m, int n, int k,
                           float alpha, const float *a, int64_t lda,
                           const float *b, int64_t ldb, float beta, float *c,
                           int64_t ldc, vs_stream_t stream) {
  return vs::sgemm_impl(variant, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0,
                        beta, c, ldc, 0, 1, static_cast<hipStream_t>(stream));
}

}  // extern "C"
