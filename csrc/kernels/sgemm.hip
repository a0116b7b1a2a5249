// Exact-fp32 SGEMM on the CDNA4 matrix cores.
//
// gfx950 has no TF32/xf32 path, but it does have an f32-in / f32-accumulate
// MFMA (v_mfma_f32_16x16x4_f32, 64 FLOP/clk/SIMD, bit-exact k-ordered fmaf
// chain) that runs at the full fp32 vector rate.  One kernel family serves
// every call: any transpose, ragged M / N / K, any alignment, strided
// batches.
//
// Operand tiles travel global -> LDS by LDS-DMA (buffer_load ... lds) into a
// three-stage ring of 16-deep k tiles.  Each operand tile is one of two LDS
// images, chosen by where K is contiguous in memory:
//   * k-rows  [rows][16] (A as stored for NN/NT, B for NT/TT): one
//     ds_read_b128 per 16-row fragment gives 4 k-steps;
//   * k-major [16][cols] (A for TN/TT, B for NN/TN): one ds_read_b32 per
//     fragment and k-step.
// NT, the reference's matrix_multiply_transposed (src/matrix.c:228-252), is
// the cheapest form: both images are k-rows.  A lane whose source lies past
// M / N / K gets an out-of-range buffer offset: the descriptor's range check
// returns zeros, so ragged edges need no separate path.  DMA = 16: 16 bytes
// per lane (contiguous dimension of both operands a multiple of 4, 16-byte
// aligned rows); DMA = 4: one float per lane for any alignment.
//
// The issue stream of the k loop is laid out by hand for two waves per SIMD
// (see Pipe below); MFMAs and fragment reads are inline asm so the interleave
// is exactly as written.
//
// Work is cut into units: whole output tiles, and -- when the tiles do not
// fill the chip evenly -- the last tiles cut into k slices whose partial
// tiles go to a workspace and are summed by a second kernel (plan_units).
// Block ids are remapped so that neighbouring tiles share an XCD's L2;
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

struct GemmArgs {
  int m, n, k;
  float alpha, beta;
  const float *a;
  int64_t lda, stride_a;
  const float *b;
  int64_t ldb, stride_b;
  float *c;
  int64_t ldc, stride_c;
  // units: tiles [0, full_tiles) are computed whole; every later tile is cut
  // into `slices` k ranges of kchunk each, whose partial tiles (dense,
  // BM x BN) go to ws[(batch * sliced_tiles + tile - full_tiles) * slices + slice]
  unsigned full_tiles, slices;
  int kchunk;
  float *ws;
};

__device__ __forceinline__ float comp(const float4 &v, int s) {
  return s == 0 ? v.x : s == 1 ? v.y : s == 2 ? v.z : v.w;
}

// Chunk swizzle of a k-rows image for 16x16 fragment reads (lanes 0-15 of a
// quarter read rows 0-15 at chunk q): conflict-free ds_read_b128 groups.
__device__ __forceinline__ int aswz4(int row, int c) { return c ^ (3 * ((row >> 3) & 1)); }

// s_waitcnt vmcnt(N) through the builtin, not inline asm: the compiler's
// wait-insertion pass understands the builtin (an asm wait is opaque to it,
// so it would add its own vmcnt(0) for every DMA it still thinks pending).
// gfx9 encoding: vmcnt[3:0] | expcnt[6:4] = 7 | lgkmcnt[11:8] = 15 | vmcnt[5:4] << 14.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt(0x0F70 | (N & 0xF) | ((N >> 4) << 14));
}

#define VS_MFMA_16X16X4(ACC, A, B) \
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(ACC) : "v"(A), "v"(B))
#define VS_MFMA_16X16X4_AGPR(ACC, A, B) \
  asm volatile("v_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+a"(ACC) : "v"(A), "v"(B))

// Tile geometry: BM x BN output tile, WM x WN waves, operand transposes, DMA
// bytes per lane, accumulators in AGPRs (a wave that owns 128 x 64 outputs
// has 128 accumulator registers: in AGPRs they leave the 128 architectural
// VGPRs of a two-waves-per-SIMD kernel to the fragments).
template <int BM_, int BN_, int WM_, int WN_, bool TA_, bool TB_, int DMA_, bool AGPR_>
struct Cfg {
  static constexpr int BM = BM_, BN = BN_, BK = 16, WM = WM_, WN = WN_;
  static constexpr int STAGES = 3;
  static constexpr bool TA = TA_, TB = TB_, AGPR = AGPR_;
  static constexpr bool AROWS = !TA, BROWS = TB;  // k-rows images
  static constexpr int DMA = DMA_;
  static constexpr int kThreads = 64 * WM * WN, kWaves = WM * WN;
  static constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  static constexpr int kImgA = BM * 64, kImgB = BN * 64, kStage = kImgA + kImgB;
  static constexpr int kLdsBytes = STAGES * kStage;
  static constexpr int kInstrBytes = 64 * DMA;  // bytes one wave instruction moves
  static constexpr int kReadsA = AROWS ? TM : 4 * TM, kReadsB = BROWS ? TN : 4 * TN;
  static constexpr int kReads = kReadsA + kReadsB;
  // loader waves (see Pipe) and the pieces (wave-wide DMA instructions) each
  // issues per tile and operand image
  static constexpr int kLoaders = kWaves == 8 ? 4 : kWaves;
  static constexpr int PA = kImgA / kInstrBytes / kLoaders;
  static constexpr int PB = kImgB / kInstrBytes / kLoaders;
  static constexpr int NP = PA + PB;
  static_assert(PA * kInstrBytes * kLoaders == kImgA && PB * kInstrBytes * kLoaders == kImgB,
                "tile not divisible into whole DMA instructions per loader wave");
  static_assert(2 * NP < 64, "vmcnt immediates");
};

constexpr uint32_t kDmaOut = 0x80000000u;  // an offset past every descriptor's range

// buffer_load_dword{,x4} ... lds of SZ bytes per lane, k advance in soffset.
// The builtin's size operand is validated against the compiling target, and
// the host pass (x86) rejects 16 -- which silently dropped the host stubs of
// every 16-byte instantiation -- so the call is compiled for the device only.
template <int SZ>
__device__ __forceinline__ void buffer_dma(__amdgpu_buffer_rsrc_t r, lds_void_t *dst,
                                           uint32_t voff, uint32_t soff) {
#if defined(__HIP_DEVICE_COMPILE__)
  if constexpr (SZ == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 16, voff, soff, 0, 0);
  else __builtin_amdgcn_raw_ptr_buffer_load_lds(r, dst, 4, voff, soff, 0, 0);
#endif
}

// LDS images, fragment registers and fragment reads of one configuration.
template <class C>
struct Tile {
  static constexpr int TM = C::TM, TN = C::TN;
  struct Frag {
    float4 a4[C::AROWS ? TM : 1];
    float a1[C::AROWS ? 1 : TM][4];
    float4 b4[C::BROWS ? TN : 1];
    float b1[C::BROWS ? 1 : TN][4];
  };
  // LDS byte offsets inside a stage of the fragment reads of lane group q
  // (fragment row / column l16 + 16 x): k-rows images put row r at 64 r
  // with the chunk swizzle (16 rows apart = 1024 B: the swizzle only depends
  // on row bit 3); k-major images put k-row kr at kr * 4 cols with a
  // column-chunk swizzle by bit 2 of kr, k-step s at + 4 s cols.  In a
  // k-major image, fragments x and x + 2 are 128 B apart, but x and x + 1
  // are not 64 B apart (the swizzle flips the chunk bit that x's parity
  // sets), so odd fragments get their own base: [0] even, [1] odd.
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
    if constexpr (R < C::kReads) {
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

  // DMA source of wave instruction J (numbered over the whole image): byte
  // offset relative to the operand's block base at k0 = 0, and the row /
  // column and k of the lane.
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

// The k loop's issue stream.
//
// Tile t lives in ring stage t % 3 and in fragment registers f[t & 1].  One
// step computes tile t from registers:
//
//   MFMA k-steps 0, 1
//   loaders: wait own DMA of tile t + 1 (counted vmcnt) ; s_barrier
//   MFMA k-steps 2, 3, with one fragment read of tile t + 1 (into the other
//   register set) behind each of the first MFMAs, then the DMA pieces of
//   tile t + 3 (into tile t's stage: every wave's reads of it retired before
//   the barrier) spread over the remaining MFMA gaps
//
// so a tile starts with its fragments already in registers and the matrix
// pipe never waits for LDS.  What keeps it busy (PMC: SQ_VALU_MFMA_BUSY 0.93
// of 4 x SQ_BUSY_CU for a burst-style loop, 0.96 here, hipBLASLt 0.98):
//   * the wave id is made uniform once (readfirstlane; threadIdx / 64 is
//     divergent to the compiler, which then wraps every M0 write in
//     v_readfirstlane), DMA voffsets are loop invariant and the k advance
//     travels in the instruction's scalar soffset: a piece is s_mov m0 +
//     v_cndmask + buffer_load ... lds, no address VALU;
//   * every step issues all its pieces: lanes at or past the end of K -- the
//     ragged part of the last tile, and whole tiles past it -- get the
//     out-of-range offset and fill their (free) stage with zeros, so the
//     counted vmcnt is the same in every step and the loop has no branch but
//     its back edge (a burst of pieces, scalar branches and address VALU
//     behind each barrier cost 3 % of the loop);
//   * with 8 waves, waves 0-3 issue the pieces of all eight.  A piece holds
//     the issuing wave for ~60 cycles, longer than the 32-cycle MFMA it
//     hides behind (ablation builds, `make ablate`: the loop runs 2 % faster
//     without the pieces, fragment reads cost 0.8 %, the barrier nothing).
//     MFMA issue goes to the older wave of a SIMD first, so waves 0-3 run
//     ahead and park at the barrier; their bubbles are filled by the younger
//     partner's MFMAs, and the partner, alone afterwards, has only LDS reads
//     between its MFMAs.
template <class C>
struct Pipe {
  using K = Tile<C>;
  static constexpr int TM = C::TM, TN = C::TN, N = 2 * TM * TN, NP = C::NP;
  // MFMA gap (index within the load half) that takes piece j
  static constexpr int slot(int j) {
    if (C::kReads + NP >= N) return N - 1 - (NP - 1 - j) % N;
    return C::kReads + (j + 1) * (N - C::kReads) / (NP + 1);
  }
  template <int I, int J, class D>
  __device__ __forceinline__ static void pieces(const D &d) {
    if constexpr (J < NP) {
      if constexpr (slot(J) == I) d(std::integral_constant<int, J>{});
      pieces<I, J + 1>(d);
    }
  }
  template <int J, class D>
  __device__ __forceinline__ static void pieces_all(const D &d) {
    if constexpr (J < NP) {
      d(std::integral_constant<int, J>{});
      pieces_all<J + 1>(d);
    }
  }
  // MFMAs of k-steps S0, S0 + 1; READ: fragment read I of the next tile
  // follows MFMA I (reads left over follow the last MFMA); DMA: so do the
  // pieces of gap I
  template <int S0, bool READ, bool DMA, class D, int I = 0>
  __device__ __forceinline__ static void half(floatx4 (&acc)[TM][TN], const typename K::Frag &f,
                                              typename K::Frag &nf, const typename K::Addr &ad,
                                              const D &d) {
    if constexpr (I < N) {
      constexpr int s = S0 + I / (TM * TN), x = (I / TN) % TM, y = I % TN;
      if constexpr (C::AGPR) VS_MFMA_16X16X4_AGPR(acc[x][y], K::opa(f, x, s), K::opb(f, y, s));
      else VS_MFMA_16X16X4(acc[x][y], K::opa(f, x, s), K::opb(f, y, s));
      if constexpr (READ && I < C::kReads) K::template read<I>(nf, ad);
      if constexpr (DMA) pieces<I, 0>(d);
      half<S0, READ, DMA, D, I + 1>(acc, f, nf, ad, d);
    } else if constexpr (READ && I < C::kReads) {
      K::template read<I>(nf, ad);
      half<S0, READ, DMA, D, I + 1>(acc, f, nf, ad, d);
    }
  }
};

// One wave's whole unit.  LOADER: this wave issues DMA pieces (pieces
// lw * PA .. + PA - 1 of the A image and likewise of B, lw = its loader
// index).  Loaders and non-loaders are separate instantiations called from a
// uniform branch, each with its own accumulators from zeroing to store
// (accumulators live across the branch made the register allocator copy /
// spill them at the join).  Every wave passes the same nk + 1 barriers.
template <class C, bool LOADER>
__device__ __forceinline__ void sgemm_run(const GemmArgs &g, uint8_t *smem, int wid) {
  using K = Tile<C>;
  using P = Pipe<C>;
  constexpr int TM = C::TM, TN = C::TN, PA = C::PA, NP = C::NP;
  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN, tiles_m = (g.m + C::BM - 1) / C::BM;
  // unit -> tile and k range
  unsigned t;
  int kb = 0, kn = g.k;
  float alpha = g.alpha, beta = g.beta;
  float *Cp;
  int64_t ldc;
  bool sliced = false;
  if (blockIdx.x < g.full_tiles) {
    t = dev::xcd_remap(blockIdx.x, g.full_tiles);
  } else {
    const unsigned u = blockIdx.x - g.full_tiles;
    t = g.full_tiles + u / g.slices;
    kb = static_cast<int>(u % g.slices) * g.kchunk;
    kn = min(g.kchunk, g.k - kb);
    sliced = true;
  }
  unsigned tm, tn;
  dev::grouped_tile(t, tiles_m, tiles_n, tm, tn);
  const int m0 = static_cast<int>(tm) * C::BM, n0 = static_cast<int>(tn) * C::BN;
  int row_lim, col_lim;  // stored rows / columns of the tile
  if (sliced) {
    const unsigned sliced_units = (tiles_m * tiles_n - g.full_tiles) * g.slices;
    Cp = g.ws + (static_cast<int64_t>(blockIdx.z) * sliced_units + (blockIdx.x - g.full_tiles)) *
                    (C::BM * C::BN);
    ldc = C::BN;
    alpha = 1.f;
    beta = 0.f;
    row_lim = C::BM;
    col_lim = C::BN;
  } else {
    ldc = g.ldc;
    Cp = g.c + blockIdx.z * g.stride_c + m0 * ldc + n0;
    row_lim = g.m - m0;
    col_lim = g.n - n0;
  }
  const int nk = (kn + C::BK - 1) / C::BK;
  const int lane = threadIdx.x & 63;
  const int wm = wid / C::WN, wn = wid % C::WN;

  // loader state: descriptors (per-block bases: A rows from m0 (k-rows) or A
  // columns from m0 (k-major), B likewise from n0, so offsets stay below
  // 2^31 for any matrix whose tile-row span fits -- checked on the host;
  // num_records covers everything, the range check only ever sees kDmaOut),
  // loop-invariant voffsets (row / column mask folded in) and k positions
  __amdgpu_buffer_rsrc_t ra, rb;
  uint32_t voa[C::PA], vob[C::PB];
  int kka[C::PA], kkb[C::PB];
  uint32_t stride_a = 0, stride_b = 0;
  uint8_t *wbase_a = nullptr, *wbase_b = nullptr;
  if constexpr (LOADER) {
    const float *Ab = g.a + blockIdx.z * g.stride_a + (C::TA ? m0 + kb * g.lda : m0 * g.lda + kb);
    const float *Bb = g.b + blockIdx.z * g.stride_b + (C::TB ? n0 * g.ldb + kb : n0 + kb * g.ldb);
    ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Ab), 0, 0x7fffffff, 0x00020000);
    rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(Bb), 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int i = 0; i < C::PA; i++) {
      const auto sa = K::template src<C::AROWS, C::BM>(wid * C::PA + i, lane, g.lda);
      voa[i] = m0 + sa.mn < g.m ? sa.off : kDmaOut;
      kka[i] = sa.kk;
    }
#pragma unroll
    for (int i = 0; i < C::PB; i++) {
      const auto sb = K::template src<C::BROWS, C::BN>(wid * C::PB + i, lane, g.ldb);
      vob[i] = n0 + sb.mn < g.n ? sb.off : kDmaOut;
      kkb[i] = sb.kk;
    }
    // k-rows images advance 16 floats per tile, k-major images 16 rows of ld
    stride_a = C::AROWS ? 64u : static_cast<uint32_t>(64 * g.lda);
    stride_b = C::BROWS ? 64u : static_cast<uint32_t>(64 * g.ldb);
    wbase_a = smem + wid * C::PA * C::kInstrBytes;
    wbase_b = smem + C::kImgA + wid * C::PB * C::kInstrBytes;
  }
  // DMA piece J of tile kt into stage st
  const auto piece_of = [&](auto jc, int st, int kt) {
    constexpr int J = decltype(jc)::value;
#if defined(VS_SGEMM_ABLATE) && (VS_SGEMM_ABLATE & 32)
    const int rem = -1;  // timing only: every lane out of range
#else
    const int rem = kn - kt * C::BK;  // <= 0 for tiles past the end
#endif
    const int ktc = min(kt, nk - 1);  // keeps soffset inside the operand
    if constexpr (J < PA) {
      const uint32_t o = kka[J] < rem ? voa[J] : kDmaOut;
      buffer_dma<C::DMA>(ra, (lds_void_t *)(wbase_a + st * C::kStage + J * C::kInstrBytes), o,
                         ktc * stride_a);
    } else {
      constexpr int j = J - PA;
      const uint32_t o = kkb[j] < rem ? vob[j] : kDmaOut;
      buffer_dma<C::DMA>(rb, (lds_void_t *)(wbase_b + st * C::kStage + j * C::kInstrBytes), o,
                         ktc * stride_b);
    }
  };
  const auto dma_all = [&](int st, int kt) {
    P::template pieces_all<0>([&](auto jc) { piece_of(jc, st, kt); });
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

  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  typename K::Offs off;
  {
    const int l16 = lane & 15, q = lane >> 4;
    off = K::offsets(wm * (C::BM / C::WM) + l16, wn * (C::BN / C::WN) + l16, q);
  }
  typename K::Frag f0, f1;

  if constexpr (LOADER) {
    dma_all(0, 0);
    dma_all(1, 1);
    dma_all(2, 2);
    wait_vmcnt<2 * NP>();
  }
  __builtin_amdgcn_s_barrier();
  K::read_all(f0, K::at(lds0, off));

  const auto nodma = [](auto) {};
  int sc = 0;  // stage of tile kt
#if defined(VS_SGEMM_ABLATE) && (VS_SGEMM_ABLATE & 4)
#define VS_SGEMM_BARRIER() (void)0
#else
#define VS_SGEMM_BARRIER() __builtin_amdgcn_s_barrier()
#endif
  // Load half of a step.  Timing-only ablations (make ablate, results are
  // wrong): 8 drops the DMA pieces, 16 the fragment reads as well.
#if defined(VS_SGEMM_ABLATE) && (VS_SGEMM_ABLATE & 16)
#define VS_SGEMM_LOADHALF(CUR, NXT) \
  P::template half<2, false, false>(acc, CUR, NXT, K::at(0u, off), nodma);
#elif defined(VS_SGEMM_ABLATE) && (VS_SGEMM_ABLATE & 8)
#define VS_SGEMM_LOADHALF(CUR, NXT) \
  P::template half<2, true, false>(acc, CUR, NXT, K::at(lds0 + sc * C::kStage, off), nodma);
#else
#define VS_SGEMM_LOADHALF(CUR, NXT)                                                 \
  P::template half<2, true, LOADER>(acc, CUR, NXT, K::at(lds0 + sc * C::kStage, off), \
                                    [&](auto jc) { piece_of(jc, st, kd); });
#endif
#define VS_SGEMM_STEP(CUR, NXT)                                                     \
  {                                                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                              \
    P::template half<0, false, false>(acc, CUR, NXT, K::at(0u, off), nodma);        \
    if constexpr (LOADER) wait_vmcnt<NP>();                                         \
    VS_SGEMM_BARRIER();                                                             \
    const int st = sc, kd = kt + 3;                                                 \
    (void)st;                                                                       \
    (void)kd;                                                                       \
    sc = sc == 2 ? 0 : sc + 1;                                                      \
    VS_SGEMM_LOADHALF(CUR, NXT)                                                     \
    kt++;                                                                           \
  }
  // The MFMA stream is straight line (no branch around it: with one, the
  // register coalescer split the accumulators and copied them at every
  // tile); the last tile's reads of the "next" tile fetch a zero-filled
  // stage and are never used.
  for (int kt = 0; kt < nk;) {
    VS_SGEMM_STEP(f0, f1)
    if (kt < nk) VS_SGEMM_STEP(f1, f0)
  }
#undef VS_SGEMM_STEP
#undef VS_SGEMM_LOADHALF
#undef VS_SGEMM_BARRIER
  // zero fills of the tiles past the end may still be in flight: LDS must
  // not be handed to the next block's waves before they land
  if constexpr (LOADER) wait_vmcnt<0>();

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
  const int arow = wm * (C::BM / C::WM) + 4 * q;   // + 16 x + r
  const int bcol = wn * (C::BN / C::WN) + l16;     // + 16 y
  const bool use_beta = beta != 0.f;
  const bool interior = row_lim >= C::BM && col_lim >= C::BN;
#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = bcol + 16 * y;
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const int row = arow + 16 * x + r;
        if (interior || (row < row_lim && col < col_lim)) {
          float *pc = Cp + static_cast<int64_t>(row) * ldc + col;
          float v = alpha * acc[x][y][r];
          if (use_beta) v += beta * *pc;
          *pc = v;
        }
      }
    }
}

template <class C>
__global__ __launch_bounds__(C::kThreads) void sgemm_kernel(GemmArgs g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t smem_gemm[];
  const int wid = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  if constexpr (C::kWaves == 8) {
    if (wid >= 4) sgemm_run<C, false>(g, smem_gemm, wid);
    else sgemm_run<C, true>(g, smem_gemm, wid);
  } else {
    sgemm_run<C, true>(g, smem_gemm, wid);
  }
}

// c tile = alpha * sum of the tile's k-slice partials + beta * c, for the
// sliced tiles [full_tiles, tiles) of every batch matrix: grid (sliced tiles
// x 1024-element chunks of a tile, batch), one float4 per lane.
template <int BM, int BN>
__global__ __launch_bounds__(256) void sgemm_slices_reduce(GemmArgs g) {
  constexpr unsigned kChunks = BM * BN / 1024;
  const unsigned tiles_n = (g.n + BN - 1) / BN, tiles_m = (g.m + BM - 1) / BM;
  const unsigned sliced = tiles_m * tiles_n - g.full_tiles;
  const unsigned st = blockIdx.x / kChunks;
  const int i = static_cast<int>((blockIdx.x % kChunks) * 256 + threadIdx.x);  // float4 in the tile
  unsigned tm, tn;
  dev::grouped_tile(g.full_tiles + st, tiles_m, tiles_n, tm, tn);
  const int row = static_cast<int>(tm) * BM + (4 * i) / BN;
  const int col = static_cast<int>(tn) * BN + (4 * i) % BN;
  if (row >= g.m || col >= g.n) return;
  const float4 *w = reinterpret_cast<const float4 *>(
      g.ws + (static_cast<int64_t>(blockIdx.y) * sliced + st) * g.slices * (BM * BN));
  float4 acc = w[i];
  for (unsigned s = 1; s < g.slices; s++) {
    const float4 v = w[s * (BM * BN / 4) + i];
    acc.x += v.x;
    acc.y += v.y;
    acc.z += v.z;
    acc.w += v.w;
  }
  float *cb = g.c + blockIdx.y * g.stride_c;
  float *pc = cb + static_cast<int64_t>(row) * g.ldc + col;
  const bool vec = (g.ldc & 3) == 0 && (reinterpret_cast<uintptr_t>(cb) & 15) == 0;
  if (vec && col + 3 < g.n) {
    float4 o{g.alpha * acc.x, g.alpha * acc.y, g.alpha * acc.z, g.alpha * acc.w};
    if (g.beta != 0.f) {
      const float4 old = *reinterpret_cast<const float4 *>(pc);
      o.x += g.beta * old.x;
      o.y += g.beta * old.y;
      o.z += g.beta * old.z;
      o.w += g.beta * old.w;
    }
    *reinterpret_cast<float4 *>(pc) = o;
  } else {
    const float v[4] = {acc.x, acc.y, acc.z, acc.w};
    for (int e = 0; e < 4 && col + e < g.n; e++)
      pc[e] = g.beta != 0.f ? g.alpha * v[e] + g.beta * pc[e] : g.alpha * v[e];
  }
}

// Whether the kernel can address this call: every DMA offset of a block
// below 2^31 bytes relative to its block base.
template <class C>
bool fits(const GemmArgs &g) {
  const int64_t ka = C::TA ? static_cast<int64_t>(g.k) * g.lda : static_cast<int64_t>(C::BM) * g.lda;
  const int64_t kb = C::TB ? static_cast<int64_t>(C::BN) * g.ldb : static_cast<int64_t>(g.k) * g.ldb;
  return g.k > 0 && 4 * (ka + 64) < (1LL << 31) && 4 * (kb + 64) < (1LL << 31);
}

template <class C>
bool launch_cfg(const GemmArgs &g, int batch, hipStream_t s) {
  if (!fits<C>(g)) return false;
  // once per instantiation (a runtime call per launch shows in host-API timings)
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(&sgemm_kernel<C>),
      hipFuncAttributeMaxDynamicSharedMemorySize, C::kLdsBytes);
  (void)attr;
  const unsigned tiles = static_cast<unsigned>(((g.m + C::BM - 1) / C::BM) *
                                               ((g.n + C::BN - 1) / C::BN));
  const unsigned units = g.full_tiles + (tiles - g.full_tiles) * g.slices;
  hipLaunchKernelGGL(sgemm_kernel<C>, dim3(units, 1, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), C::kLdsBytes, s, g);
  if (g.full_tiles < tiles)
    hipLaunchKernelGGL((sgemm_slices_reduce<C::BM, C::BN>),
                       dim3((tiles - g.full_tiles) * (C::BM * C::BN / 1024),
                            static_cast<unsigned>(batch)),
                       dim3(256), 0, s, g);
  return true;
}

// Tile geometry x transposes.
template <int BM, int BN, int WM, int WN, int DMA, bool AGPR>
bool launch_t(const GemmArgs &g, int ta, int tb, int batch, hipStream_t s) {
  if (!ta && !tb) return launch_cfg<Cfg<BM, BN, WM, WN, false, false, DMA, AGPR>>(g, batch, s);
  if (!ta && tb) return launch_cfg<Cfg<BM, BN, WM, WN, false, true, DMA, AGPR>>(g, batch, s);
  if (ta && !tb) return launch_cfg<Cfg<BM, BN, WM, WN, true, false, DMA, AGPR>>(g, batch, s);
  return launch_cfg<Cfg<BM, BN, WM, WN, true, true, DMA, AGPR>>(g, batch, s);
}

// 16-byte DMA needs 16-byte aligned operand rows whose contiguous dimension
// (k for k-rows images, m / n for k-major ones) is a multiple of 4.
bool dma16(const GemmArgs &g, int ta, int tb, int batch) {
  const auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int ca = ta ? g.m : g.k, cb = tb ? g.k : g.n;
  return al(g.a) && al(g.b) && g.lda % 4 == 0 && g.ldb % 4 == 0 && ca % 4 == 0 &&
         cb % 4 == 0 && (batch == 1 || (g.stride_a % 4 == 0 && g.stride_b % 4 == 0));
}

// Tiles: 0 = 64 x 64 (4 waves of 32 x 32), 1 = 128 x 128 (8 waves of
// 64 x 32), 2 = 256 x 256 (8 waves of 128 x 64, AGPR accumulators; 16-byte
// DMA only: with 4-byte pieces a tile would overrun the vmcnt range).
constexpr int kTileDim[3] = {64, 128, 256};

bool launch_tile(const GemmArgs &g, int ta, int tb, int batch, hipStream_t s, int tile, bool d16) {
  if (tile == 2) return launch_t<256, 256, 2, 4, 16, true>(g, ta, tb, batch, s);
  if (tile == 1) {
    if (d16) return launch_t<128, 128, 2, 4, 16, false>(g, ta, tb, batch, s);
    return launch_t<128, 128, 2, 4, 4, false>(g, ta, tb, batch, s);
  }
  if (d16) return launch_t<64, 64, 2, 2, 16, false>(g, ta, tb, batch, s);
  return launch_t<64, 64, 2, 2, 4, false>(g, ta, tb, batch, s);
}

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

// How one tile size cuts a call into units, and the modelled time.
struct Units {
  unsigned full, slices;
  int kchunk;
  double cost;  // in 256 x 256 x 16 tile steps per CU
};

// Work distribution for `tiles` output tiles per matrix (x batch) of
// dim x dim over the chip.  Whole tiles run first; when the last round would
// leave CUs idle (r = tiles mod CUs tiles on CUs CUs), those r tiles are cut
// into floor(CUs / r) k slices each (>= kMinSlice deep), so the tail round
// costs 1 / slices of a tile instead of a whole one, plus a reduction pass
// over the r tiles.  With fewer tiles than CUs this is plain split-K.
// Batched calls are only sliced when all their tiles together under-fill
// the chip.
// Cost model, in steps of one 256 x 256 x 16 tile on one CU (3.4 us).  The
// busiest CU gets n = ceil(units / CUs) units and runs them in waves of up
// to `resident` co-resident blocks; a wave of c blocks of ks k-tiles costs
// c x (ks + kEpilogue) x area / rate(c) plus the start-up latency, where
// rate(c) is the measured per-CU throughput of the tile size relative to
// 256 x 256: a lone 64 x 64 block (one wave per SIMD) reaches 0.57, four
// sharing the CU 0.85.  The reduction pass costs a launch plus its bytes at
// HBM speed.  Predictions are within ~5 % of measured times from 300 x 1000 x
// 256 to 8192^3 (profiles/r3/sgemm/model_fit.md).
Units plan_units(long tiles, int batch, int k, int dim, bool allow_slices) {
  constexpr int kMinSlice = 128, kMaxSlices = 16;
  constexpr double kStepUs = 3.41, kLatencyUs = 2.5, kEpilogue = 2.0, kReduceUs = 4.0,
                   kReduceBytesPerUs = 3.0e6;
  static const double rate_full[3] = {0.85, 0.975, 1.0}, rate_alone[3] = {0.57, 0.90, 1.0};
  static const int resident[3] = {4, 2, 1};  // blocks sharing a CU
  const long cus = device_cu_count();
  const int ti = dim == 64 ? 0 : dim == 128 ? 1 : 2;
  const double area = static_cast<double>(dim) * dim / 65536.0;
  const auto rate = [&](long c) {
    const int res = resident[ti];
    if (res == 1 || c >= res) return rate_full[ti];
    return rate_alone[ti] + (rate_full[ti] - rate_alone[ti]) * (c - 1) / (res - 1);
  };
  const auto units_cost = [&](long units, int ks) {  // equal units of ks k-tiles over the chip
    if (units == 0) return 0.0;
    const long n = (units + cus - 1) / cus;
    const double work = (ks + kEpilogue) * area;
    const long full = n / resident[ti], c = n % resident[ti];
    double t = full * (resident[ti] * work / rate(resident[ti]) + kLatencyUs / kStepUs);
    if (c) t += c * work / rate(c) + kLatencyUs / kStepUs;
    return t;
  };
  const int ks = (k + 15) / 16;
  const long total = tiles * batch;
  const long rounds = total / cus, r = total % cus;
  Units u{static_cast<unsigned>(tiles), 1, 0, units_cost(total, ks)};
  if (!allow_slices || r == 0 || (batch > 1 && rounds > 0)) return u;
  long s = std::min<long>(std::min<long>(cus / r, k / kMinSlice), kMaxSlices);
  if (s < 2) return u;
  const int kchunk = static_cast<int>(((k + s - 1) / s + 15) / 16 * 16);
  s = (k + kchunk - 1) / kchunk;
  if (s < 2) return u;
  const double reduce_us = kReduceUs + static_cast<double>(r) * (s + 1) * dim * dim * 4 /
                                           kReduceBytesPerUs;
  const double cost = units_cost(total - r, ks) + units_cost(r * s, kchunk / 16) +
                      reduce_us / kStepUs;
  if (cost >= u.cost) return u;
  const long sliced_tiles = batch > 1 ? tiles : r;  // batch > 1: rounds == 0, every tile
  u.full = static_cast<unsigned>(tiles - sliced_tiles);
  u.slices = static_cast<unsigned>(s);
  u.kchunk = kchunk;
  u.cost = cost;
  return u;
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
  GemmArgs g{m, n, k, alpha, beta, a, lda, sa, b, ldb, sb, c, ldc, sc, 0, 1, 0, nullptr};
  if (variant < 0) variant = default_variant();
  VS_REQUIRE(variant < VS_SGEMM_VARIANTS, "vs_sgemm: unknown variant %d (0..%d)", variant,
             VS_SGEMM_VARIANTS - 1);
  const bool d16 = dma16(g, ta, tb, batch);
  // variant: tile + 3 * (1 = whole tiles only); default: best modelled tile
  int tile = -1;
  bool allow_slices = true;
  if (variant >= 0) {
    tile = variant % 3;
    allow_slices = variant < 3;
    if (tile == 2 && !d16) tile = 1;
  }
  Units units{};
  const auto plan = [&](int ti) {
    const int dim = kTileDim[ti];
    const long tiles = static_cast<long>((m + dim - 1) / dim) * ((n + dim - 1) / dim);
    return plan_units(tiles, batch, k, dim, allow_slices);
  };
  if (tile >= 0) {
    units = plan(tile);
  } else {
    for (int ti = d16 ? 2 : 1; ti >= 0; ti--) {  // larger tiles win ties
      const Units u = plan(ti);
      if (tile < 0 || u.cost < units.cost * 0.999) {
        units = u;
        tile = ti;
      }
    }
  }
  const auto ws_floats = [&](const Units &u) {
    const int dim = kTileDim[tile];
    const long tiles = static_cast<long>((m + dim - 1) / dim) * ((n + dim - 1) / dim);
    return static_cast<size_t>(tiles - u.full) * u.slices * dim * dim * batch;
  };
  // inside a stream capture large scratch is not available: whole tiles only
  if (units.slices > 1 && scratch_refused_in_capture(sizeof(float) * ws_floats(units), s)) {
    allow_slices = false;
    units = plan(tile);
  }
  g.full_tiles = units.full;
  g.slices = units.slices;
  g.kchunk = units.kchunk;
  DeviceBuffer ws;
  if (units.slices > 1) {
    VS_TRY(ws.alloc(sizeof(float) * ws_floats(units), s));
    g.ws = ws.as<float>();
  }
  const bool ok = launch_tile(g, ta, tb, batch, s, tile, d16);
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
// include/simd/gpu.h; negative: the default selection).
vs_status vs_sgemm_variant(int variant, int ta, int tb, int m, int n, int k,
                           float alpha, const float *a, int64_t lda,
                           const float *b, int64_t ldb, float beta, float *c,
                           int64_t ldc, vs_stream_t stream) {
  return vs::sgemm_impl(variant, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0,
                        beta, c, ldc, 0, 1, static_cast<hipStream_t>(stream));
}

// Batched form of the tuning entry point.
vs_status vs_sgemm_variant_batched(int variant, int ta, int tb, int m, int n, int k,
                                   float alpha, const float *a, int64_t lda, int64_t sa,
                                   const float *b, int64_t ldb, int64_t sb, float beta,
                                   float *c, int64_t ldc, int64_t sc, int batch,
                                   vs_stream_t stream) {
  return vs::sgemm_impl(variant, ta, tb, m, n, k, alpha, a, lda, sa, b, ldb, sb,
                        beta, c, ldc, sc, batch, static_cast<hipStream_t>(stream));
}

}  // extern "C"
