// bf16 matrix-core GEMM and the "bf16x3" fast-fp32 mode.
//
//   vs_gemm_bf16:   C(fp32) = alpha op(A) op(B) + beta C, A/B bf16.
//   vs_sgemm_ex(VS_GEMM_BF16X3, ...): fp32 operands split as x = hi + lo
//     (hi = bf16(x), lo = bf16(x - hi)); C = hi_a hi_b + hi_a lo_b + lo_a hi_b
//     accumulated in fp32 by v_mfma_f32_32x32x16_bf16.  The dropped lo*lo
//     term and the 16-bit split leave ~2^-16 relative error per product
//     (vs 2^-24 for exact fp32) at 3 bf16 MFMAs (3 x 32 cycles per 32x32x16
//     block) instead of 8 f32 MFMAs (8 x 64 cycles) -- a 5x shorter MFMA
//     critical path.
//
// Structure: a prepass (split_kernel / pack_kernel) writes every operand as
// a zero-padded, K-contiguous bf16 image ([Mp][Kp] for A, [Np][Kp] for B,
// transposing B when it is stored [k][n]); a bf16 operand already stored
// K-contiguous with whole tiles is read in place.  The main kernel
// (gemm_glds_kernel) stages both images global -> LDS with
// global_load_lds_dwordx4 into two XOR-swizzled stages and runs
// v_mfma_f32_16x16x32_bf16 on 256 x 256 (bf16) / 256 x 128 (bf16x3) tiles,
// or v_mfma_f32_32x32x16_bf16 on 128 x 128 tiles when the large ones cannot
// fill every CU.  (Earlier
// register-staged, three/four-stage ring and transposed-read variants were
// measured slower or spilled and are in git history,
// profiles/r1/gemm_modes_v*.log.)
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
namespace gbf {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));


__device__ __forceinline__ uint16_t bf16_bits(float x) {
  const __bf16 h = static_cast<__bf16>(x);
  return __builtin_bit_cast(uint16_t, h);
}
__device__ __forceinline__ float bf16_float(uint16_t b) {
  return __uint_as_float(static_cast<uint32_t>(b) << 16);
}

// ---------------------------------------------------------------- prepass
// dst[r][c] (r < rows_p, c < cols_p, row stride cols_p) from the logical
// operand element (r, c) = src[r * ld + c] (TRANS = 0) or src[c * ld + r]
// (TRANS = 1), zero outside rows x cols.  SPLIT: fp32 source, writes hi and
// lo images; else bf16 source (uint16 bits), one image.  64 x 64 tiles, one
// 8-element chunk per thread and step: 16-byte loads along the source's
// contiguous dimension (VEC: ld, the batch stride and the base are 8-element
// aligned) and 16-byte stores along c; TRANS turns the tile round through a
// [64][65] float LDS image (conflict-free both ways).  Rows of the source
// that end inside a chunk fall back to guarded scalar loads.
template <bool SPLIT>
__device__ __forceinline__ void load8(const void *src, int64_t off, bool vec, int lim,
                                      int64_t step, float (&v)[8]) {
  if (vec && lim >= 8) {
    if (SPLIT) {
      const float4 *p = reinterpret_cast<const float4 *>(static_cast<const float *>(src) + off);
      const float4 x = p[0], y = p[1];
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
    } else {
      const uint4 x = *reinterpret_cast<const uint4 *>(static_cast<const uint16_t *>(src) + off);
      const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int j = 0; j < 4; j++) {
        v[2 * j] = __uint_as_float(w[j] << 16);
        v[2 * j + 1] = __uint_as_float(w[j] & 0xffff0000u);
      }
    }
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const int64_t o = off + j * step;
    v[j] = j < lim ? (SPLIT ? static_cast<const float *>(src)[o]
                            : bf16_float(static_cast<const uint16_t *>(src)[o]))
                   : 0.f;
  }
}

template <bool SPLIT>
__device__ __forceinline__ void store8(uint16_t *hi, uint16_t *lo, int64_t o, const float (&v)[8]) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint16_t h0 = bf16_bits(v[2 * j]), h1 = bf16_bits(v[2 * j + 1]);
    h[j] = h0 | (static_cast<uint32_t>(h1) << 16);
    if (SPLIT)
      l[j] = bf16_bits(v[2 * j] - bf16_float(h0)) |
             (static_cast<uint32_t>(bf16_bits(v[2 * j + 1] - bf16_float(h1))) << 16);
  }
  *reinterpret_cast<uint4 *>(hi + o) = make_uint4(h[0], h[1], h[2], h[3]);
  if (SPLIT) *reinterpret_cast<uint4 *>(lo + o) = make_uint4(l[0], l[1], l[2], l[3]);
}

template <bool SPLIT, bool TRANS>
__global__ __launch_bounds__(256) void pack_kernel(const void *__restrict__ src,
                                                   int64_t ld, int rows, int cols,
                                                   int rows_p, int cols_p,
                                                   uint16_t *__restrict__ hi,
                                                   uint16_t *__restrict__ lo,
                                                   int64_t sstride, int64_t dstride, bool vec) {
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int sub = threadIdx.x >> 3, ch = (threadIdx.x & 7) * 8;  // 32 x 8 chunks
  const int64_t sb = blockIdx.z * sstride, db = blockIdx.z * dstride;
  if (TRANS) {
    __shared__ float tile[64][65];  // [c][r]
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int c = c0 + sub + 32 * i, r = r0 + ch;  // 8 consecutive r of source row c
      float v[8];
      load8<SPLIT>(src, sb + static_cast<int64_t>(c) * ld + r, vec,
                   c < cols ? rows - r : 0, 1, v);
#pragma unroll
      for (int j = 0; j < 8; j++) tile[sub + 32 * i][ch + j] = v[j];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int r = r0 + sub + 32 * i, c = c0 + ch;
      if (r >= rows_p || c >= cols_p) continue;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; j++) v[j] = tile[ch + j][sub + 32 * i];
      store8<SPLIT>(hi, lo, db + static_cast<int64_t>(r) * cols_p + c, v);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int r = r0 + sub + 32 * i, c = c0 + ch;
      if (r >= rows_p || c >= cols_p) continue;
      float v[8];
      load8<SPLIT>(src, sb + static_cast<int64_t>(r) * ld + c, vec,
                   r < rows ? cols - c : 0, 1, v);
      store8<SPLIT>(hi, lo, db + static_cast<int64_t>(r) * cols_p + c, v);
    }
  }
}

// ------------------------------------------------------------ main kernel
struct Args {
  const uint16_t *a[2];  // [Mp][Kp] images: hi (and lo)
  const uint16_t *b[2];  // [Np][Kp]
  int64_t sa, sb;        // batch strides of the images (elements)
  int64_t lda, ldb;      // row strides of the images (elements; >= kp)
  int kp;                // K extent (a multiple of the k tile)
  int m, n;              // logical output size
  float alpha, beta;
  float *c;
  int64_t ldc, sc;
  int stagger;           // the two waves of a SIMD issue their DMA half a tile apart
};

// Pack one operand.  rows x cols is the logical op(X) with rows along the
// output (M or N) and cols along K; `trans` = element (r, c) at src[c*ld + r].
vs_status pack(bool split, bool trans, const void *src, int64_t ld, int rows, int cols,
               int rows_p, int cols_p, uint16_t *hi, uint16_t *lo, int64_t sstride,
               int batch, hipStream_t s) {
  // rows_p, cols_p are multiples of the tile sizes (>= 32), so every 8-chunk
  // of the destination is either wholly inside or wholly outside
  const dim3 grid(static_cast<unsigned>((cols_p + 63) / 64),
                  static_cast<unsigned>((rows_p + 63) / 64), static_cast<unsigned>(batch));
  const int64_t dstride = static_cast<int64_t>(rows_p) * cols_p;
  const bool vec = ld % 8 == 0 && (batch == 1 || sstride % 8 == 0) &&
                   reinterpret_cast<uintptr_t>(src) % 16 == 0;
  if (split && trans)
    hipLaunchKernelGGL((pack_kernel<true, true>), grid, dim3(256), 0, s, src, ld, rows, cols,
                       rows_p, cols_p, hi, lo, sstride, dstride, vec);
  else if (split)
    hipLaunchKernelGGL((pack_kernel<true, false>), grid, dim3(256), 0, s, src, ld, rows, cols,
                       rows_p, cols_p, hi, lo, sstride, dstride, vec);
  else if (trans)
    hipLaunchKernelGGL((pack_kernel<false, true>), grid, dim3(256), 0, s, src, ld, rows, cols,
                       rows_p, cols_p, hi, lo, sstride, dstride, vec);
  else
    hipLaunchKernelGGL((pack_kernel<false, false>), grid, dim3(256), 0, s, src, ld, rows,
                       cols, rows_p, cols_p, hi, lo, sstride, dstride, vec);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// ------------------------------------------- LDS-DMA (glds) pipelined kernel
// Large problems: operand tiles go global -> LDS with global_load_lds_dwordx4
// (no VGPR round trip, 1 KiB per wave-instruction, LDS destination
// wave-uniform base + 16 * lane), two LDS stages, the next k-tile's DMA
// issued before the current tile's MFMAs and retired by one vmcnt(0) +
// barrier per k-tile.  LDS images are [row][BK] bf16 with 16-byte chunk c
// of row r stored at chunk c ^ ((r / S) & (NC - 1)) (S rows share a 256-byte
// bank row): the XOR is applied to the per-lane SOURCE address of the DMA
// and to the fragment read, so the 16-lane groups of ds_read_b128 hit 16
// distinct bank groups (cdna_hip_programming.md §5.4 rule 21, T2).
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glob_void;

template <int TERMS_, int BM_, int BN_, int BK_, int WM_, int WN_>
struct GCfg {
  static constexpr int TERMS = TERMS_, BM = BM_, BN = BN_, BK = BK_, WM = WM_, WN = WN_;
  static constexpr int NIMG = TERMS == 1 ? 1 : 2;
  static constexpr int kThreads = 64 * WM * WN, kWaves = WM * WN;
  static constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static constexpr int NC = BK / 8;        // 16-byte chunks per row
  static constexpr int RB = BK * 2;        // row bytes
  static constexpr int S = 256 / RB;       // rows per 256-byte bank row
  static constexpr int RPI = 1024 / RB;    // rows per glds wave-instruction
  static constexpr int kImgA = BM * RB, kImgB = BN * RB;  // bytes
  static constexpr int kStage = NIMG * (kImgA + kImgB);
  static constexpr int kLdsBytes = 2 * kStage;
  static constexpr int kInstrA = kImgA / 1024 / kWaves;   // per wave, per image
  static constexpr int kInstrB = kImgB / 1024 / kWaves;
  static_assert(kInstrA * 1024 * kWaves == kImgA && kInstrB * 1024 * kWaves == kImgB,
                "image not divisible into whole glds instructions per wave");
  static_assert(BK % 16 == 0 && RB <= 1024, "BK");
};

template <class C>
__device__ __forceinline__ int swz(int row, int c) {
  return c ^ ((row / C::S) & (C::NC - 1));
}

// DMA one image tile (ROWS x BK at row0, k0) into the LDS image at `dst`.
template <class C, int INSTR>
__device__ __forceinline__ void dma_image(const uint16_t *__restrict__ img, int64_t ld,
                                          int row0, int k0, uint8_t *dst, int wave,
                                          int lane) {
#pragma unroll
  for (int i = 0; i < INSTR; i++) {
    const int j = wave * INSTR + i;            // instruction index in the image
    const int row = j * C::RPI + lane / C::NC;  // tile row this lane fills
    const int pc = lane % C::NC;                // physical chunk it fills
    const int c = swz<C>(row, pc);              // logical chunk stored there
    const uint16_t *src = img + static_cast<int64_t>(row0 + row) * ld + k0 + 8 * c;
    __builtin_amdgcn_global_load_lds((glob_void *)const_cast<uint16_t *>(src),
                                     (lds_void *)(dst + j * 1024), 16, 0, 0);
  }
}

template <class C>
__device__ __forceinline__ bf16x8 gfrag(const uint8_t *img, int row, int c) {
  return *reinterpret_cast<const bf16x8 *>(img + row * C::RB + swz<C>(row, c) * 16);
}

typedef float floatx4 __attribute__((ext_vector_type(4)));

// M16: v_mfma_f32_16x16x32_bf16 on 16 x 16 blocks (32-deep steps) instead of
// v_mfma_f32_32x32x16_bf16 on 32 x 32 blocks (16-deep steps): the same
// fragment reads and accumulator registers per wave.
template <class C, bool M16 = false>
__global__ __launch_bounds__(C::kThreads) void gemm_glds_kernel(Args g) {
  extern __shared__ __attribute__((aligned(1024))) uint8_t glds_lds[];
  constexpr int TM = C::TM, TN = C::TN, NI = C::NIMG;
  const unsigned tiles_m = (g.m + C::BM - 1) / C::BM;
  const unsigned tiles_n = (g.n + C::BN - 1) / C::BN;
  const unsigned ntiles = tiles_m * tiles_n;
  unsigned tile = blockIdx.x;  // the M16 form walks tiles blockIdx.x, + gridDim.x, ...
  int m0, n0;
  const auto place = [&] {
    unsigned tm, tn;
    dev::grouped_tile(dev::xcd_remap(tile, ntiles), tiles_m, tiles_n, tm, tn);
    m0 = static_cast<int>(tm) * C::BM;
    n0 = static_cast<int>(tn) * C::BN;
  };
  place();
  const uint16_t *A[2], *B[2];
#pragma unroll
  for (int i = 0; i < NI; i++) {
    A[i] = g.a[i] + blockIdx.z * g.sa;
    B[i] = g.b[i] + blockIdx.z * g.sb;
  }
  float *Cp = g.c + blockIdx.z * g.sc;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid / C::WN, wn = wid % C::WN;
  const int lrow = lane & 31, lh = lane >> 5;
  const int arow = wm * (C::BM / C::WM) + lrow;
  const int brow = wn * (C::BN / C::WN) + lrow;

  auto img_a = [&](int buf, int i) { return glds_lds + buf * C::kStage + i * C::kImgA; };
  auto img_b = [&](int buf, int i) {
    return glds_lds + buf * C::kStage + NI * C::kImgA + i * C::kImgB;
  };
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int i = 0; i < NI; i++) {
      dma_image<C, C::kInstrA>(A[i], g.lda, m0, k0, img_a(buf, i), wid, lane);
      dma_image<C, C::kInstrB>(B[i], g.ldb, n0, k0, img_b(buf, i), wid, lane);
    }
  };

  const int nk = g.kp / C::BK;
  const bool use_beta = g.beta != 0.f;
  if constexpr (M16) {
    constexpr int XM = 2 * TM, XN = 2 * TN;  // 16 x 16 blocks per wave
    const int l16 = lane & 15, lq = lane >> 4;
    const int arow16 = wm * (C::BM / C::WM) + l16, brow16 = wn * (C::BN / C::WN) + l16;
    floatx4 acc[XM][XN];
    for (;;) {
#pragma unroll
      for (int i = 0; i < XM; i++)
#pragma unroll
        for (int j = 0; j < XN; j++) acc[i][j] = floatx4{0.f, 0.f, 0.f, 0.f};
      stage(0, 0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      // The two waves of a SIMD (wave i and i + 4) issue their share of the next
      // tile's DMA at different times -- waves 0-3 before the tile's MFMAs, waves
      // 4-7 a quarter of the tile later -- so one of them runs MFMAs
      // while the other pays the DMA issue cost (60-185 cycles per piece).
      const bool late = g.stagger && wid >= C::kWaves / 2;
      for (int kt = 0; kt < nk; kt++) {
        const int cur = kt & 1;
        if (!late && kt + 1 < nk) stage(cur ^ 1, (kt + 1) * C::BK);
#pragma unroll
        for (int ks = 0; ks < C::BK / 32; ks++) {
          const int c = 4 * ks + lq;
          bf16x8 fa[NI][XM], fb[NI][XN];
#pragma unroll
          for (int i = 0; i < NI; i++) {
#pragma unroll
            for (int x = 0; x < XM; x++) fa[i][x] = gfrag<C>(img_a(cur, i), arow16 + 16 * x, c);
#pragma unroll
            for (int y = 0; y < XN; y++) fb[i][y] = gfrag<C>(img_b(cur, i), brow16 + 16 * y, c);
          }
#pragma unroll
          for (int x = 0; x < XM; x++) {
            // a quarter of the tile's MFMAs in: the late waves' DMA
            if (ks == 0 && x == XM / 2 && late && kt + 1 < nk) stage(cur ^ 1, (kt + 1) * C::BK);
#pragma unroll
            for (int y = 0; y < XN; y++) {
              if (C::TERMS == 3) {
                acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[1][x], fb[0][y], acc[x][y],
                                                                    0, 0, 0);
                acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][x], fb[1][y], acc[x][y],
                                                                    0, 0, 0);
              }
              acc[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[0][x], fb[0][y], acc[x][y], 0,
                                                                  0, 0);
            }
          }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      // C through LDS: a 16 x 16 block leaves lane l with rows 4 (l / 16) + r of
      // column l % 16, i.e. 64-byte row segments and one dword store per value
      // (4096 dword stores per wave).  Each wave turns 32 rows
      // x 64 columns at a time round through its own LDS patch (row stride 68
      // floats: conflict-free both ways) and stores float4 per lane, 256-byte
      // row segments.
      const bool vec = (g.ldc & 3) == 0 && (g.sc & 3) == 0 &&
                       (reinterpret_cast<uintptr_t>(g.c) & 15) == 0;
      if (vec) {
        constexpr int LDW = 68, WN64 = C::BN / C::WN;  // patch row stride (floats); wave tile width
        static_assert(WN64 == 64, "the patch is 64 columns wide");
        float *patch = reinterpret_cast<float *>(glds_lds) + wid * 32 * LDW;
        const int wrow0 = m0 + wm * (C::BM / C::WM), wcol0 = n0 + wn * WN64;
#pragma unroll
        for (int p = 0; p < XM / 2; p++) {
#pragma unroll
          for (int xx = 0; xx < 2; xx++)
#pragma unroll
            for (int y = 0; y < XN; y++)
#pragma unroll
              for (int r = 0; r < 4; r++)
                patch[(16 * xx + 4 * lq + r) * LDW + 16 * y + l16] =
                    g.alpha * acc[2 * p + xx][y][r];
#pragma unroll
          for (int i = 0; i < 8; i++) {
            const int pr = 4 * i + lq, pc4 = 4 * l16;
            const floatx4 v = *reinterpret_cast<const floatx4 *>(patch + pr * LDW + pc4);
            const int row = wrow0 + 32 * p + pr, col = wcol0 + pc4;
            if (row >= g.m || col >= g.n) continue;
            float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
            if (col + 3 < g.n) {
              floatx4 o = v;
              if (use_beta) o += g.beta * *reinterpret_cast<const floatx4 *>(pc);
              *reinterpret_cast<floatx4 *>(pc) = o;
            } else {
#pragma unroll
              for (int e = 0; e < 4; e++)
                if (col + e < g.n) pc[e] = use_beta ? v[e] + g.beta * pc[e] : v[e];
            }
          }
        }
      } else {
        // 16 x 16 block: lane l holds rows 4 (l / 16) + r, column l % 16
#pragma unroll
        for (int x = 0; x < XM; x++)
#pragma unroll
          for (int y = 0; y < XN; y++) {
            const int col = n0 + brow16 + 16 * y;
            if (col >= g.n) continue;
#pragma unroll
            for (int r = 0; r < 4; r++) {
              const int row = m0 + arow16 - l16 + 16 * x + 4 * lq + r;
              if (row < g.m) {
                float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
                float v = g.alpha * acc[x][y][r];
                if (use_beta) v += g.beta * *pc;
                *pc = v;
              }
            }
          }
      }
      tile += gridDim.x;
      if (tile >= ntiles) return;
      place();
      __syncthreads();  // the LDS patches are read before the next tile's DMA lands on them
    }
  }

  floatx16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; i++)
#pragma unroll
    for (int j = 0; j < TN; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    if (kt + 1 < nk) stage(cur ^ 1, (kt + 1) * C::BK);
#pragma unroll
    for (int ks = 0; ks < C::BK / 16; ks++) {
      const int c = 2 * ks + lh;
      bf16x8 fa[NI][TM], fb[NI][TN];
#pragma unroll
      for (int i = 0; i < NI; i++) {
#pragma unroll
        for (int x = 0; x < TM; x++) fa[i][x] = gfrag<C>(img_a(cur, i), arow + 32 * x, c);
#pragma unroll
        for (int y = 0; y < TN; y++) fb[i][y] = gfrag<C>(img_b(cur, i), brow + 32 * y, c);
      }
#pragma unroll
      for (int x = 0; x < TM; x++)
#pragma unroll
        for (int y = 0; y < TN; y++) {
          if (C::TERMS == 3) {
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][x], fb[0][y],
                                                                acc[x][y], 0, 0, 0);
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][x], fb[1][y],
                                                                acc[x][y], 0, 0, 0);
          }
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][x], fb[0][y],
                                                              acc[x][y], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

#pragma unroll
  for (int x = 0; x < TM; x++)
#pragma unroll
    for (int y = 0; y < TN; y++) {
      const int col = n0 + brow + 32 * y;
      if (col >= g.n) continue;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = m0 + arow - lrow + 32 * x + (r & 3) + 8 * (r >> 2) + 4 * lh;
        if (row < g.m) {
          float *pc = Cp + static_cast<int64_t>(row) * g.ldc + col;
          float v = g.alpha * acc[x][y][r];
          if (use_beta) v += g.beta * *pc;
          *pc = v;
        }
      }
    }
}

template <class C, bool M16 = false>
vs_status launch_glds(const Args &g, int batch, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute(
      reinterpret_cast<const void *>(&gemm_glds_kernel<C, M16>),
      hipFuncAttributeMaxDynamicSharedMemorySize, C::kLdsBytes);  // once per instantiation
  VS_HIP(attr);
  const unsigned tiles = static_cast<unsigned>(((g.m + C::BM - 1) / C::BM) *
                                               ((g.n + C::BN - 1) / C::BN));
  // g.stagger & 2: the 16 x 16 x 32 form as one workgroup per CU walking the tiles
  const unsigned grid = M16 && (g.stagger & 2)
                            ? std::min(tiles, static_cast<unsigned>(device_cu_count())) : tiles;
  hipLaunchKernelGGL((gemm_glds_kernel<C, M16>), dim3(grid, 1, static_cast<unsigned>(batch)),
                     dim3(C::kThreads), C::kLdsBytes, s, g);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

using G1 = GCfg<1, 256, 256, 64, 2, 4>;   // bf16: 128 KiB LDS, 8 waves of 128 x 64
using G3 = GCfg<3, 256, 128, 32, 4, 2>;   // bf16x3: 96 KiB LDS, 8 waves of 64 x 64
using G1S = GCfg<1, 128, 128, 64, 2, 2>;  // bf16, small problems: 64 KiB, 4 waves of 64 x 64
using G3S = GCfg<3, 128, 128, 32, 2, 2>;  // bf16x3, small problems: 64 KiB

int env_variant() {
  static const int v = [] {
    const char *e = std::getenv("VELES_GEMM_BF16_VARIANT");
    return e && *e ? std::atoi(e) : -1;
  }();
  return v;
}

vs_status gemm_impl(bool split, int ta, int tb, int m, int n, int k, float alpha,
                    const void *a, int64_t lda, int64_t sa, const void *b, int64_t ldb,
                    int64_t sb, float beta, float *c, int64_t ldc, int64_t sc, int batch,
                    int variant, hipStream_t s) {
  VS_REQUIRE(m >= 0 && n >= 0 && k >= 0 && batch >= 0, "gemm_bf16: negative dimension");
  if (m == 0 || n == 0 || batch == 0) return VS_OK;
  VS_REQUIRE(a && b && c, "gemm_bf16: null pointer");
  VS_REQUIRE(ldc >= n, "gemm_bf16: ldc < n");
  VS_REQUIRE(lda >= (ta ? m : k) && ldb >= (tb ? k : n), "gemm_bf16: leading dimension too small");
  if (batch > kMaxGridY) {
    const size_t es = split ? sizeof(float) : sizeof(uint16_t);
    return batch_chunks(batch, [&](long long b0, int nb) {
      return gemm_impl(split, ta, tb, m, n, k, alpha,
                       static_cast<const char *>(a) + b0 * sa * es, lda, sa,
                       static_cast<const char *>(b) + b0 * sb * es, ldb, sb, beta,
                       c + b0 * sc, ldc, sc, nb, variant, s);
    });
  }
  if (variant < 0) variant = env_variant();
  if (variant < 0) {
    // large tiles once they fill every CU, else 128 x 128
    const long tl = static_cast<long>((m + G1::BM - 1) / G1::BM) * ((n + G1::BN - 1) / G1::BN) *
                    batch;
    variant = tl >= 256 ? 2 : 0;  // the large tiles run 6 % faster on the 16 x 16 x 32 shape
  }
  VS_REQUIRE(variant >= 0 && variant <= 4, "gemm_bf16: unknown variant %d (0..4)", variant);
  // The wave pairs of the bf16 large tile issue their DMA a quarter of a tile apart
  // (4096^3: 1205 -> 1301 TFLOP/s, 8192^3: 1238 -> 1307; the 32-deep bf16x3 tiles lose with
  // it: 371 -> 305); variant 4 is variant 2 without it and without the tile walk (A/B arm).
  // bit 0: staggered DMA issue; bit 1: one workgroup per CU walks the tiles (+2 % on the bf16
  // large tile: no workgroup turnaround between tiles; the bf16x3 tiles lose with it)
  const int stagger = variant == 2 && !split ? 3 : 0;
  if (variant == 4) variant = 2;
  // 0 / 1: small / large tiles on v_mfma_f32_32x32x16_bf16; 2 / 3: large / small tiles on
  // v_mfma_f32_16x16x32_bf16
  const bool m16 = variant >= 2;
  variant = variant == 2 ? 1 : variant == 3 ? 0 : variant;
  const int bm = variant == 1 ? (split ? G3::BM : G1::BM) : (split ? G3S::BM : G1S::BM);
  const int bn = variant == 1 ? (split ? G3::BN : G1::BN) : (split ? G3S::BN : G1S::BN);
  const int bk = variant == 1 ? (split ? G3::BK : G1::BK) : (split ? G3S::BK : G1S::BK);
  const int mp = (m + bm - 1) / bm * bm, np = (n + bn - 1) / bn * bn;
  const int kp = k == 0 ? bk : (k + bk - 1) / bk * bk;
  const int ni = split ? 2 : 1;
  // A bf16 operand already stored K-contiguous ([rows][ld]: A unless ta, B
  // when tb) with whole tiles and aligned rows is read in place -- no
  // prepass, no workspace (VELES_GEMM_BF16_PACK=1 forces the copy).
  static const bool force_pack = [] {
    const char *e = std::getenv("VELES_GEMM_BF16_PACK");
    return e && *e == '1';
  }();
  const auto direct = [&](bool kcontig, int rows, int rows_p, const void *p, int64_t ld,
                          int64_t st) {
    return !split && !force_pack && kcontig && rows == rows_p && k == kp && ld % 8 == 0 &&
           (batch == 1 || st % 8 == 0) && reinterpret_cast<uintptr_t>(p) % 16 == 0;
  };
  const bool da = direct(ta == 0, m, mp, a, lda, sa);
  const bool db = direct(tb != 0, n, np, b, ldb, sb);
  const size_t ea = static_cast<size_t>(mp) * kp, eb = static_cast<size_t>(np) * kp;
  const size_t wa = da ? 0 : ea * ni * batch, wb = db ? 0 : eb * ni * batch;
  DeviceBuffer buf;
  if (wa + wb) VS_TRY(buf.alloc((wa + wb) * sizeof(uint16_t), s));
  uint16_t *pa = da ? nullptr : buf.as<uint16_t>();
  uint16_t *pb = db ? nullptr : buf.as<uint16_t>() + wa;
  Args g{};
  // A: logical (M x K), element (r, c) at a[r*lda + c] unless ta.
  if (da) {
    g.a[0] = static_cast<const uint16_t *>(a);
    g.sa = batch == 1 ? 0 : sa;
    g.lda = lda;
  } else {
    VS_TRY(pack(split, ta != 0, a, lda, m, k, mp, kp, pa, split ? pa + ea * batch : nullptr,
                sa, batch, s));
    g.a[0] = pa;
    g.a[1] = split ? pa + ea * batch : nullptr;
    g.sa = static_cast<int64_t>(ea);
    g.lda = kp;
  }
  // B: logical op(B)^T (N x K): element (n, k) at b[k*ldb + n] unless tb.
  if (db) {
    g.b[0] = static_cast<const uint16_t *>(b);
    g.sb = batch == 1 ? 0 : sb;
    g.ldb = ldb;
  } else {
    VS_TRY(pack(split, tb == 0, b, ldb, n, k, np, kp, pb, split ? pb + eb * batch : nullptr,
                sb, batch, s));
    g.b[0] = pb;
    g.b[1] = split ? pb + eb * batch : nullptr;
    g.sb = static_cast<int64_t>(eb);
    g.ldb = kp;
  }
  g.kp = kp;
  g.m = m;
  g.n = n;
  g.alpha = alpha;
  g.beta = beta;
  g.c = c;
  g.ldc = ldc;
  g.sc = sc;
  g.stagger = stagger;
  if (m16 && variant == 1)
    return split ? launch_glds<G3, true>(g, batch, s) : launch_glds<G1, true>(g, batch, s);
  if (m16) return split ? launch_glds<G3S, true>(g, batch, s) : launch_glds<G1S, true>(g, batch, s);
  if (variant == 1) return split ? launch_glds<G3>(g, batch, s) : launch_glds<G1>(g, batch, s);
  return split ? launch_glds<G3S>(g, batch, s) : launch_glds<G1S>(g, batch, s);
}

}  // namespace
}  // namespace gbf
}  // namespace vs

using namespace vs;

extern "C" {

vs_status vs_gemm_bf16(int ta, int tb, int m, int n, int k, float alpha, const uint16_t *a,
                       int64_t lda, const uint16_t *b, int64_t ldb, float beta, float *c,
                       int64_t ldc, vs_stream_t stream) {
  clear_error();
  return gbf::gemm_impl(false, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0, beta, c, ldc, 0, 1,
                        -1, static_cast<hipStream_t>(stream));
}

vs_status vs_gemm_bf16_variant(int variant, int ta, int tb, int m, int n, int k, float alpha,
                               const uint16_t *a, int64_t lda, const uint16_t *b,
                               int64_t ldb, float beta, float *c, int64_t ldc,
                               vs_stream_t stream) {
  clear_error();
  return gbf::gemm_impl(false, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0, beta, c, ldc, 0, 1,
                        variant, static_cast<hipStream_t>(stream));
}

vs_status vs_gemm_bf16_strided_batched(int ta, int tb, int m, int n, int k, float alpha,
                                       const uint16_t *a, int64_t lda, int64_t sa,
                                       const uint16_t *b, int64_t ldb, int64_t sb,
                                       float beta, float *c, int64_t ldc, int64_t sc,
                                       int batch, vs_stream_t stream) {
  clear_error();
  return gbf::gemm_impl(false, ta, tb, m, n, k, alpha, a, lda, sa, b, ldb, sb, beta, c, ldc, sc,
                        batch, -1, static_cast<hipStream_t>(stream));
}

vs_status vs_sgemm_bf16x3(int ta, int tb, int m, int n, int k, float alpha, const float *a,
                          int64_t lda, const float *b, int64_t ldb, float beta, float *c,
                          int64_t ldc, int variant, vs_stream_t stream) {
  clear_error();
  return gbf::gemm_impl(true, ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0, beta, c, ldc, 0, 1,
                        variant, static_cast<hipStream_t>(stream));
}

vs_status vs_sgemm_bf16x3_strided_batched(int ta, int tb, int m, int n, int k, float alpha,
                                          const float *a, int64_t lda, int64_t sa,
                                          const float *b, int64_t ldb, int64_t sb, float beta,
                                          float *c, int64_t ldc, int64_t sc, int batch,
                                          vs_stream_t stream) {
  clear_error();
  return gbf::gemm_impl(true, ta, tb, m, n, k, alpha, a, lda, sa, b, ldb, sb, beta, c, ldc, sc,
                        batch, -1, static_cast<hipStream_t>(stream));
}

}  // extern "C"
