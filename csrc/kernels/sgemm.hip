// Exact-fp32 SGEMM on the CDNA4 matrix cores.
//
// gfx950 has no TF32/xf32 path, but it does have an f32-in / f32-accumulate
// MFMA (v_mfma_f32_32x32x2_f32, 64 FLOP/clk/SIMD, bit-exact k-ordered fmaf
// chain) that runs at the full fp32 vector rate while leaving the VALU free
// for addressing and staging (cdna_hip_programming.md §3 'FP32-input MFMA').
//
// Structure (per workgroup, 256 threads = 4 waves):
//   * output tile BM x BN = 128 x 128, each wave a 64 x 64 quadrant held as
//     2 x 2 accumulators of 32 x 32 (64 accumulator registers);
//   * K is walked in BK = 16 steps through two LDS buffers laid out k-major
//     ([k][m], [k][n], rows padded to 132 floats), so an MFMA operand is one
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
// stack-copied B column, no blocking) and :53-65 / :67-80 (scalar).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "csrc/kernels/device.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int kThreads = 256;
constexpr int LDP = 132;  // LDS row pitch (floats): 128 + 4 keeps 16-B rows

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

// Loads this thread's share of one BK x 128 operand tile into registers.
//   KCONTIG: operand stored [mn][k] (k contiguous) -> 2 float4 along k.
//   else   : operand stored [k][mn] (mn contiguous) -> 2 float4 along mn.
template <bool KCONTIG, bool VEC>
__device__ __forceinline__ void load_tile(const float *__restrict__ p,
                                          int64_t ld, int mn0, int mn_lim,
                                          int k0, int k_lim, float4 (&r)[2]) {
#pragma unroll
  for (int l = 0; l < 2; l++) {
    const int idx = threadIdx.x + l * kThreads;
    int mn, kk;
    if (KCONTIG) {
      mn = mn0 + (idx >> 2);
      kk = k0 + (idx & 3) * 4;
    } else {
      kk = k0 + (idx >> 5);
      mn = mn0 + (idx & 31) * 4;
    }
    float v[4];
    const float *base = KCONTIG ? p + mn * ld + kk : p + kk * ld + mn;
    const bool full = KCONTIG ? (mn < mn_lim && kk + 3 < k_lim)
                              : (kk < k_lim && mn + 3 < mn_lim);
    if (VEC && full) {
      const float4 t = *reinterpret_cast<const float4 *>(base);
      v[0] = t.x;
      v[1] = t.y;
      v[2] = t.z;
      v[3] = t.w;
    } else {
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const bool ok = KCONTIG ? (mn < mn_lim && kk + c < k_lim)
                                : (kk < k_lim && mn + c < mn_lim);
        v[c] = ok ? base[c] : 0.f;
      }
    }
    r[l] = make_float4(v[0], v[1], v[2], v[3]);
  }
}

template <bool KCONTIG>
__device__ __forceinline__ void store_tile(float *__restrict__ s,
                                           const float4 (&r)[2]) {
#pragma unroll
  for (int l = 0; l < 2; l++) {
    const int idx = threadIdx.x + l * kThreads;
    if (KCONTIG) {
      const int mn = idx >> 2, kq = (idx & 3) * 4;
      s[(kq + 0) * LDP + mn] = r[l].x;
      s[(kq + 1) * LDP + mn] = r[l].y;
      s[(kq + 2) * LDP + mn] = r[l].z;
      s[(kq + 3) * LDP + mn] = r[l].w;
    } else {
      const int kk = idx >> 5, mn = (idx & 31) * 4;
      *reinterpret_cast<float4 *>(s + kk * LDP + mn) = r[l];
    }
  }
}

// TA / TB: operand stored transposed relative to op().  A is KCONTIG unless
// TA; B is KCONTIG only if TB.
template <bool TA, bool TB, bool VEC>
__global__ __launch_bounds__(kThreads) void sgemm_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][BK * LDP];

  const unsigned tiles_n = (g.n + BN - 1) / BN;
  const unsigned tiles_m = (g.m + BM - 1) / BM;
  const unsigned ntiles = tiles_m * tiles_n;
  const unsigned t = dev::xcd_remap(blockIdx.x, ntiles);
  const int tm = static_cast<int>(t / tiles_n), tn = static_cast<int>(t % tiles_n);
  const int m0 = tm * BM, n0 = tn * BN;

  const float *A = g.a + blockIdx.z * g.stride_a;
  const float *B = g.b + blockIdx.z * g.stride_b;
  float *C = g.c + blockIdx.z * g.stride_c;

  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int lrow = lane & 31, lk = lane >> 5;

  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++)
#pragma unroll
      for (int r = 0; r < 16; r++) acc[i][j][r] = 0.f;

  float4 ra[2], rb[2];
  const int nk = (g.k + BK - 1) / BK;

  load_tile<!TA, VEC>(A, g.lda, m0, g.m, 0, g.k, ra);
  load_tile<TB, VEC>(B, g.ldb, n0, g.n, 0, g.k, rb);
  store_tile<!TA>(lds[0][0], ra);
  store_tile<TB>(lds[0][1], rb);
  __syncthreads();

  for (int kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile<!TA, VEC>(A, g.lda, m0, g.m, (kt + 1) * BK, g.k, ra);
      load_tile<TB, VEC>(B, g.ldb, n0, g.n, (kt + 1) * BK, g.k, rb);
    }
    const float *As = lds[cur][0];
    const float *Bs = lds[cur][1];
#pragma unroll
    for (int s = 0; s < BK / 2; s++) {
      const int kr = 2 * s + lk;
      float fa[2], fb[2];
#pragma unroll
      for (int i = 0; i < 2; i++) fa[i] = As[kr * LDP + wm * 64 + i * 32 + lrow];
#pragma unroll
      for (int j = 0; j < 2; j++) fb[j] = Bs[kr * LDP + wn * 64 + j * 32 + lrow];
#pragma unroll
      for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(fa[i], fb[j],
                                                           acc[i][j], 0, 0, 0);
    }
    if (more) {
      store_tile<!TA>(lds[cur ^ 1][0], ra);
      store_tile<TB>(lds[cur ^ 1][1], rb);
    }
    __syncthreads();
  }

  // Epilogue: C/D map of the 32x32 f32 MFMA: col = lane & 31,
  // row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5).
  const bool use_beta = g.beta != 0.f;
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) {
      const int col = n0 + wn * 64 + j * 32 + lrow;
      if (col >= g.n) continue;
#pragma unroll
      for (int r = 0; r < 16; r++) {
        const int row = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < g.m) {
          float *pc = C + static_cast<int64_t>(row) * g.ldc + col;
          float v = g.alpha * acc[i][j][r];
          if (use_beta) v += g.beta * *pc;
          *pc = v;
        }
      }
    }
}

template <bool TA, bool TB>
void launch_t(const GemmArgs &g, bool vec, dim3 grid, hipStream_t s) {
  if (vec)
    hipLaunchKernelGGL((sgemm_kernel<TA, TB, true>), grid, dim3(kThreads), 0, s, g);
  else
    hipLaunchKernelGGL((sgemm_kernel<TA, TB, false>), grid, dim3(kThreads), 0, s, g);
}

vs_status sgemm_impl(int ta, int tb, int m, int n, int k, float alpha,
                     const float *a, int64_t lda, int64_t sa, const float *b,
                     int64_t ldb, int64_t sb, float beta, float *c, int64_t ldc,
                     int64_t sc, int batch, hipStream_t s) {
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
  const unsigned tiles =
      static_cast<unsigned>(((m + BM - 1) / BM) * ((n + BN - 1) / BN));
  const dim3 grid(tiles, 1, static_cast<unsigned>(batch));
  if (!ta && !tb) launch_t<false, false>(g, vec, grid, s);
  else if (!ta && tb) launch_t<false, true>(g, vec, grid, s);
  else if (ta && !tb) launch_t<true, false>(g, vec, grid, s);
  else launch_t<true, true>(g, vec, grid, s);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // namespace
}  // namespace vs

extern "C" {

vs_status vs_sgemm(int ta, int tb, int m, int n, int k, float alpha,
                   const float *a, int64_t lda, const float *b, int64_t ldb,
                   float beta, float *c, int64_t ldc, vs_stream_t stream) {
  return vs::sgemm_impl(ta, tb, m, n, k, alpha, a, lda, 0, b, ldb, 0, beta, c,
                        ldc, 0, 1, static_cast<hipStream_t>(stream));
}

vs_status vs_sgemm_strided_batched(int ta, int tb, int m, int n, int k,
                                   float alpha, const float *a, int64_t lda,
                                   int64_t sa, const float *b, int64_t ldb,
                                   int64_t sb, float beta, float *c,
                                   int64_t ldc, int64_t sc, int batch,
                                   vs_stream_t stream) {
  return vs::sgemm_impl(ta, tb, m, n, k, alpha, a, lda, sa, b, ldb, sb, beta,
                        c, ldc, sc, batch, static_cast<hipStream_t>(stream));
}

}  // extern "C"
