// Radix-16/8/4/2 Stockham FFT for CDNA4 (replaces the
// reference's external FFTF, reference src/convolve.c:131-143).
//
//   * n <= 16384: one workgroup per signal (several per workgroup for small
//     n), the whole signal in LDS, 16 points per thread, see fft_core.h;
//   * n up to 2^24: four-step decomposition n = N1 x N2 -- N1-point column
//     transforms over 16+ adjacent columns per workgroup (so every global
//     access is a >= 128-byte segment) with the inter-step twiddle fused in,
//     N2-point row transforms, and a tiled transpose to natural order;
//   * real transforms (n real <-> n/2+1 complex, the FFTF_TYPE_REAL layout of
//     n+2 floats) are an n/2-point complex transform of the even/odd-packed
//     signal plus one split/merge pass.
// Twiddles are tabulated in double precision on the host (one float2 per
// root), so transforms are accurate to a few ulp of the output norm.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <cmath>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "csrc/kernels/fft_core.h"
#include "csrc/kernels/fft_plan.h"
#include "csrc/runtime/runtime.h"
#include "simd/gpu.h"

namespace vs {
namespace fft {

// ------------------------------------------------------------ twiddle cache
namespace {

std::mutex g_tw_mu;
std::map<std::pair<int, int>, float2 *> g_tw;        // (device, logn)
std::map<std::pair<int, int>, float2 *> g_tw_split;  // (device, logn)

inline float2 root(long long m, long long n) {
  // exp(-2 pi i m / n) in double, reduced to the first octant for accuracy.
  const double a = -2.0 * M_PI * static_cast<double>(m) / static_cast<double>(n);
  return make_float2(static_cast<float>(std::cos(a)), static_cast<float>(std::sin(a)));
}

const float2 *upload(std::vector<float2> &host, vs_status *st) {
  void *d = nullptr;
  if (hipMalloc(&d, host.size() * sizeof(float2)) != hipSuccess ||
      hipMemcpy(d, host.data(), host.size() * sizeof(float2),
                hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipGetLastError();
    set_error("FFT plan: cannot upload %zu twiddles", host.size());
    *st = VS_ERR_ALLOC;
    return nullptr;
  }
  *st = VS_OK;
  return static_cast<float2 *>(d);
}

}  // namespace

const float2 *twiddles(int logn, vs_status *st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(g_tw_mu);
  auto key = std::make_pair(dev, logn);
  auto it = g_tw.find(key);
  if (it != g_tw.end()) {
    *st = VS_OK;
    return it->second;
  }
  const long long n = 1LL << logn;
  std::vector<float2> host(n);
  for (long long m = 0; m < n; m++) host[m] = root(m, n);
  const float2 *d = upload(host, st);
  if (d) g_tw[key] = const_cast<float2 *>(d);
  return d;
}

const float2 *split_twiddles(int logn, vs_status *st) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(g_tw_mu);
  auto key = std::make_pair(dev, logn);
  auto it = g_tw_split.find(key);
  if (it != g_tw_split.end()) {
    *st = VS_OK;
    return it->second;
  }
  const long long n = 1LL << logn;
  const int s = split_shift(logn);
  const long long nlo = 1LL << s, nhi = n >> s;
  std::vector<float2> host(nlo + nhi);
  for (long long r = 0; r < nlo; r++) host[r] = root(r, n);
  for (long long q = 0; q < nhi; q++) host[nlo + q] = root(q << s, n);
  const float2 *d = upload(host, st);
  if (d) g_tw_split[key] = const_cast<float2 *>(d);
  return d;
}

int ilog2_exact(long long n) {
  if (n <= 0 || (n & (n - 1))) return -1;
  int l = 0;
  while ((1LL << l) < n) l++;
  return l;
}

// ------------------------------------------------------------- kernels
namespace {

template <int LOGN>
struct LdsGeom {
  using PL = Plan<LOGN>;
  static constexpr int SPB = PL::TPS >= 256 ? 1 : 256 / PL::TPS;  // signals/block
  static constexpr int kThreads = PL::TPS * SPB;
};

template <int LOGN, bool INV>
__global__ __launch_bounds__(LdsGeom<LOGN>::kThreads) void c2c_lds_kernel(
    const float2 *__restrict__ in, float2 *__restrict__ out, int batch,
    const float2 *__restrict__ tw) {
  using PL = Plan<LOGN>;
  constexpr int SPB = LdsGeom<LOGN>::SPB;
  __shared__ float2 lds[SPB * PL::kLds];
  const int sl = threadIdx.x / PL::TPS, t = threadIdx.x % PL::TPS;
  const long long sig = static_cast<long long>(blockIdx.x) * SPB + sl;
  const bool active = sig < batch;
  const float2 *src = in + sig * PL::N;
  float2 v[PL::E];
  constexpr int R0 = PL::first_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
    for (int j = 0; j < R0; j++)
      v[b * R0 + j] = active ? src[reg_index<PL, R0>(t, b, j)] : make_float2(0.f, 0.f);
  transform<PL, INV, false>(v, lds + sl * PL::kLds, t, tw);
  if (!active) return;
  float2 *dst = out + sig * PL::N;
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++) dst[reg_index<PL, RL>(t, b, j)] = v[b * RL + j];
}

template <int LOG1>
struct ColGeom {
  using PL = Plan<LOG1>;
  // <= 512 threads: at 1024 (LOG1 = 10, 16 columns) the 128-VGPR budget of
  // 4 waves/SIMD spilled the 16-point-per-thread working set.
  static constexpr int COLS = PL::TPS >= 64 ? 512 / PL::TPS : (PL::TPS >= 16 ? 16 : 256 / PL::TPS);
  static constexpr int kThreads = PL::TPS * COLS;
};

__device__ __forceinline__ float2 split_root(const float2 *__restrict__ tws,
                                             int s, long long a) {
  const long long nlo = 1LL << s;
  return cmul(tws[nlo + (a >> s)], tws[a & (nlo - 1)]);
}

// Column pass of the four-step FFT (see launch_cols).
template <int LOG1, bool INV>
__global__ __launch_bounds__(ColGeom<LOG1>::kThreads) void cols_kernel(
    const float2 *__restrict__ in, float2 *__restrict__ out, int log2n2,
    const float2 *__restrict__ tw1, const float2 *__restrict__ tws, int s) {
  using PL = Plan<LOG1>;
  constexpr int COLS = ColGeom<LOG1>::COLS;
  __shared__ float2 lds[COLS * PL::kLds];
  const long long n2 = 1LL << log2n2;
  const long long N = n2 << LOG1;
  const int cl = threadIdx.x % COLS, t = threadIdx.x / COLS;
  const long long col = static_cast<long long>(blockIdx.x) * COLS + cl;
  const float2 *src = in + blockIdx.y * N + col;
  float2 *dst = out + blockIdx.y * N + col;
  float2 v[PL::E];
  constexpr int R0 = PL::first_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
    for (int j = 0; j < R0; j++) {
      const int k1 = reg_index<PL, R0>(t, b, j);
      float2 x = src[static_cast<long long>(k1) * n2];
      if (INV) x = cmulc(x, split_root(tws, s, col * k1));
      v[b * R0 + j] = x;
    }
  transform<PL, INV, false>(v, lds + cl * PL::kLds, t, tw1);
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++) {
      const int k1 = reg_index<PL, RL>(t, b, j);
      float2 x = v[b * RL + j];
      if (!INV) x = cmul(x, split_root(tws, s, col * k1));
      dst[static_cast<long long>(k1) * n2] = x;
    }
}

// out[sig][c][r] = in[sig][r][c] for an R x C matrix (R = 2^logr).
__global__ __launch_bounds__(256) void transpose_kernel(
    const float2 *__restrict__ in, float2 *__restrict__ out, int logr, int logc) {
  __shared__ float2 tile[32][33];
  const long long R = 1LL << logr, C = 1LL << logc;
  const float2 *src = in + blockIdx.z * R * C;
  float2 *dst = out + blockIdx.z * R * C;
  const long long r0 = static_cast<long long>(blockIdx.y) * 32;
  const long long c0 = static_cast<long long>(blockIdx.x) * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const long long r = r0 + ty + k, c = c0 + tx;
    if (r < R && c < C) tile[ty + k][tx] = src[r * C + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 32; k += 8) {
    const long long c = c0 + ty + k, r = r0 + tx;
    if (r < R && c < C) dst[c * R + r] = tile[tx][ty + k];
  }
}

// Split (forward) / merge (inverse) pass of the real transforms.
//   forward: Z = FFT_{n/2}(x as complex) -> X[k], k = 0..n/2
//   inverse: X[k], k = 0..n/2 -> Z for IFFT_{n/2} (unnormalised convention)
__global__ __launch_bounds__(256) void r2c_post_kernel(
    const float2 *__restrict__ z, float2 *__restrict__ X, int logh, int batch,
    const float2 *__restrict__ tw) {  // tw: exp(-2 pi i m / n), n = 2^(logh+1)
  const int h = 1 << logh;
  const long long total = static_cast<long long>(batch) * (h / 2 + 1);
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total;
       g += static_cast<long long>(gridDim.x) * 256) {
    const long long sig = g / (h / 2 + 1);
    const int k = static_cast<int>(g % (h / 2 + 1));  // handles k and h - k
    const float2 *zs = z + sig * h;
    float2 *xs = X + sig * (h + 1);
    const float2 a = zs[k & (h - 1)];
    const float2 b = zs[(h - k) & (h - 1)];
    // E = (a + conj b)/2, O = (a - conj b)/(2i); X[k] = E + W^k O
    const float2 e = make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
    const float2 o = make_float2(0.5f * (a.y + b.y), -0.5f * (a.x - b.x));
    const float2 w = tw[k];
    const float2 wo = cmul(w, o);
    xs[k] = cadd(e, wo);
    // X[h - k] = conj(E) + W^(h-k) conj(O) = conj(E - W^k O)
    if (k != 0 && k != h - k) xs[h - k] = make_float2(e.x - wo.x, -(e.y - wo.y));
    if (k == 0) xs[h] = make_float2(e.x - o.x, e.y - o.y);  // W^h = -1
  }
}

__global__ __launch_bounds__(256) void c2r_pre_kernel(
    const float2 *__restrict__ X, float2 *__restrict__ z, int logh, int batch,
    const float2 *__restrict__ tw) {
  const int h = 1 << logh;
  const long long total = static_cast<long long>(batch) * h;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total;
       g += static_cast<long long>(gridDim.x) * 256) {
    const long long sig = g / h;
    const int k = static_cast<int>(g % h);
    const float2 *xs = X + sig * (h + 1);
    const float2 a = xs[k];
    const float2 c = xs[h - k];
    const float2 bh = make_float2(c.x, -c.y);  // X[k + h] = conj X[h - k]
    const float2 e = cadd(a, bh);
    const float2 o = cmulc(csub(a, bh), tw[k]);  // (X[k]-X[k+h]) W^-k
    // Z = E + i O
    z[sig * h + k] = make_float2(e.x - o.y, e.y + o.x);
  }
}

template <int LOGN>
void launch_lds_t(bool inv, const float2 *in, float2 *out, int batch,
                  const float2 *tw, hipStream_t s) {
  using G = LdsGeom<LOGN>;
  const unsigned grid = static_cast<unsigned>((batch + G::SPB - 1) / G::SPB);
  if (inv)
    hipLaunchKernelGGL((c2c_lds_kernel<LOGN, true>), dim3(grid), dim3(G::kThreads),
                       0, s, in, out, batch, tw);
  else
    hipLaunchKernelGGL((c2c_lds_kernel<LOGN, false>), dim3(grid), dim3(G::kThreads),
                       0, s, in, out, batch, tw);
}

template <int LOG1>
void launch_cols_t(bool inv, const float2 *in, float2 *out, int log2n2,
                   int batch, const float2 *tw1, const float2 *tws, int sh,
                   hipStream_t s) {
  using G = ColGeom<LOG1>;
  const dim3 grid(static_cast<unsigned>((1LL << log2n2) / G::COLS),
                  static_cast<unsigned>(batch));
  if (inv)
    hipLaunchKernelGGL((cols_kernel<LOG1, true>), grid, dim3(G::kThreads), 0, s,
                       in, out, log2n2, tw1, tws, sh);
  else
    hipLaunchKernelGGL((cols_kernel<LOG1, false>), grid, dim3(G::kThreads), 0, s,
                       in, out, log2n2, tw1, tws, sh);
}


// ----------------------------------------- fused four-step FFT convolution
// conv_four_step: the whole-signal FFT convolution (filters longer than an
// overlap-save block) in three passes over the data instead of seven:
//   cols_pack_kernel   real signal pairs (2p, 2p+1) -> z, forward column FFT
//                      with twiddles (replaces pack + cols);
//   rows_conv_kernel   row FFT -> x H (same permuted layout) -> inverse row
//                      FFT with reversed radices, in registers / LDS
//                      (replaces rows + multiply + inverse rows);
//   cols_unpack_kernel inverse column FFT -> scaled outputs of both signals
//                      straight to y (replaces inverse cols + unpack).
template <int LOG1>
__global__ __launch_bounds__(ColGeom<LOG1>::kThreads) void cols_pack_kernel(
    const float *__restrict__ x, int xlen, int64_t xs, int batch, float2 *__restrict__ out,
    int log2n2, const float2 *__restrict__ tw1, const float2 *__restrict__ tws, int s) {
  using PL = Plan<LOG1>;
  constexpr int COLS = ColGeom<LOG1>::COLS;
  __shared__ float2 lds[COLS * PL::kLds];
  const long long n2 = 1LL << log2n2;
  const long long N = n2 << LOG1;
  const int cl = threadIdx.x % COLS, t = threadIdx.x / COLS;
  const long long col = static_cast<long long>(blockIdx.x) * COLS + cl;
  const long long s0 = 2LL * blockIdx.y, s1 = s0 + 1;
  const float *x0 = x + s0 * xs;
  const float *x1 = x + (s1 < batch ? s1 : s0) * xs;
  const bool has1 = s1 < batch;
  float2 *dst = out + blockIdx.y * N + col;
  float2 v[PL::E];
  constexpr int R0 = PL::first_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
    for (int j = 0; j < R0; j++) {
      const long long n = static_cast<long long>(reg_index<PL, R0>(t, b, j)) * n2 + col;
      const bool in = n < xlen;
      v[b * R0 + j] = make_float2(in ? x0[n] : 0.f, in && has1 ? x1[n] : 0.f);
    }
  transform<PL, false, false>(v, lds + cl * PL::kLds, t, tw1);
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++) {
      const int k1 = reg_index<PL, RL>(t, b, j);
      dst[static_cast<long long>(k1) * n2] = cmul(v[b * RL + j], split_root(tws, s, col * k1));
    }
}

// One row (n2 = 2^LOG2 points, contiguous) per workgroup: forward FFT,
// times H of the same row, inverse FFT with the radices reversed so the
// spectrum never leaves the registers between the two transforms.
template <int LOG2>
__global__ __launch_bounds__(Plan<LOG2>::TPS) void rows_conv_kernel(
    float2 *__restrict__ z, const float2 *__restrict__ H, int log1, const float2 *__restrict__ tw) {
  using PL = Plan<LOG2>;
  __shared__ float2 lds[PL::kLds];
  const int t = threadIdx.x;
  const long long rows = 1LL << log1;
  const long long row = blockIdx.x;                  // row within the pair's matrix
  float2 *zr = z + (static_cast<long long>(blockIdx.y) * rows + row) * PL::N;
  const float2 *hr = H + row * PL::N;
  float2 v[PL::E];
  constexpr int R0 = PL::first_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
    for (int j = 0; j < R0; j++) v[b * R0 + j] = zr[reg_index<PL, R0>(t, b, j)];
  __builtin_amdgcn_sched_barrier(0);
  transform<PL, false, false>(v, lds, t, tw);
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++)
      v[b * RL + j] = cmul(v[b * RL + j], hr[reg_index<PL, RL>(t, b, j)]);
  transform<PL, true, true>(v, lds, t, tw);
  constexpr int RI = PL::radix(0);
#pragma unroll
  for (int b = 0; b < PL::E / RI; b++)
#pragma unroll
    for (int j = 0; j < RI; j++) zr[reg_index<PL, RI>(t, b, j)] = v[b * RI + j];
}

template <int LOG1>
__global__ __launch_bounds__(ColGeom<LOG1>::kThreads) void cols_unpack_kernel(
    const float2 *__restrict__ in, int log2n2, int batch, float *__restrict__ y, int64_t ys,
    int ylen, float scale, const float2 *__restrict__ tw1, const float2 *__restrict__ tws,
    int s) {
  using PL = Plan<LOG1>;
  constexpr int COLS = ColGeom<LOG1>::COLS;
  __shared__ float2 lds[COLS * PL::kLds];
  const long long n2 = 1LL << log2n2;
  const long long N = n2 << LOG1;
  const int cl = threadIdx.x % COLS, t = threadIdx.x / COLS;
  const long long col = static_cast<long long>(blockIdx.x) * COLS + cl;
  const float2 *src = in + blockIdx.y * N + col;
  const long long s0 = 2LL * blockIdx.y, s1 = s0 + 1;
  float *y0 = y + s0 * ys;
  float *y1 = y + s1 * ys;
  const bool has1 = s1 < batch;
  float2 v[PL::E];
  constexpr int R0 = PL::first_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / R0; b++)
#pragma unroll
    for (int j = 0; j < R0; j++) {
      const int k1 = reg_index<PL, R0>(t, b, j);
      v[b * R0 + j] = cmulc(src[static_cast<long long>(k1) * n2], split_root(tws, s, col * k1));
    }
  transform<PL, true, false>(v, lds + cl * PL::kLds, t, tw1);
  constexpr int RL = PL::last_radix(false);
#pragma unroll
  for (int b = 0; b < PL::E / RL; b++)
#pragma unroll
    for (int j = 0; j < RL; j++) {
      const long long n = static_cast<long long>(reg_index<PL, RL>(t, b, j)) * n2 + col;
      if (n < ylen) {
        y0[n] = v[b * RL + j].x * scale;
        if (has1) y1[n] = v[b * RL + j].y * scale;
      }
    }
}

template <int LOG1>
void launch_pack_t(const float *x, int xlen, int64_t xs, int batch, float2 *z, int log2n2,
                   const float2 *tw1, const float2 *tws, int sh, hipStream_t s) {
  using G = ColGeom<LOG1>;
  const dim3 grid(static_cast<unsigned>((1LL << log2n2) / G::COLS),
                  static_cast<unsigned>((batch + 1) / 2));
  hipLaunchKernelGGL((cols_pack_kernel<LOG1>), grid, dim3(G::kThreads), 0, s, x, xlen, xs,
                     batch, z, log2n2, tw1, tws, sh);
}

template <int LOG1>
void launch_unpack_t(const float2 *z, int log2n2, int batch, float *y, int64_t ys, int ylen,
                     float scale, const float2 *tw1, const float2 *tws, int sh, hipStream_t s) {
  using G = ColGeom<LOG1>;
  const dim3 grid(static_cast<unsigned>((1LL << log2n2) / G::COLS),
                  static_cast<unsigned>((batch + 1) / 2));
  hipLaunchKernelGGL((cols_unpack_kernel<LOG1>), grid, dim3(G::kThreads), 0, s, z, log2n2,
                     batch, y, ys, ylen, scale, tw1, tws, sh);
}

template <int LOG2>
void launch_rows_conv_t(float2 *z, const float2 *H, int log1, int npairs, const float2 *tw,
                        hipStream_t s) {
  hipLaunchKernelGGL((rows_conv_kernel<LOG2>), dim3(1u << log1, static_cast<unsigned>(npairs)),
                     dim3(Plan<LOG2>::TPS), 0, s, z, H, log1, tw);
}
}  // namespace

vs_status launch_c2c_lds(int logn, bool inv, const float2 *in, float2 *out,
                         int batch, hipStream_t s) {
  VS_REQUIRE(logn >= 1 && logn <= kMaxLdsLog, "LDS FFT: log2 n = %d out of range", logn);
  if (batch <= 0) return VS_OK;
  vs_status st;
  const float2 *tw = twiddles(logn, &st);
  if (!tw) return st;
  switch (logn) {
#define VS_CASE(L) \
  case L: launch_lds_t<L>(inv, in, out, batch, tw, s); break;
    VS_CASE(1) VS_CASE(2) VS_CASE(3) VS_CASE(4) VS_CASE(5) VS_CASE(6) VS_CASE(7)
    VS_CASE(8) VS_CASE(9) VS_CASE(10) VS_CASE(11) VS_CASE(12) VS_CASE(13) VS_CASE(14)
#undef VS_CASE
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status launch_cols(int logn, bool inv, const float2 *in, float2 *out,
                      int batch, hipStream_t s) {
  int log1, log2;
  four_step_split(logn, &log1, &log2);
  VS_REQUIRE(log1 >= 1 && log1 <= 10, "four-step: bad split of 2^%d", logn);
  vs_status st;
  const float2 *tw1 = twiddles(log1, &st);
  if (!tw1) return st;
  const float2 *tws = split_twiddles(logn, &st);
  if (!tws) return st;
  const int sh = split_shift(logn);
  switch (log1) {
#define VS_CASE(L) \
  case L: launch_cols_t<L>(inv, in, out, log2, batch, tw1, tws, sh, s); break;
    VS_CASE(1) VS_CASE(2) VS_CASE(3) VS_CASE(4) VS_CASE(5)
    VS_CASE(6) VS_CASE(7) VS_CASE(8) VS_CASE(9) VS_CASE(10)
#undef VS_CASE
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status launch_transpose(int log1, int log2, const float2 *in, float2 *out,
                           int batch, hipStream_t s) {
  const dim3 grid(static_cast<unsigned>(((1LL << log2) + 31) / 32),
                  static_cast<unsigned>(((1LL << log1) + 31) / 32),
                  static_cast<unsigned>(batch));
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, s, in, out, log1, log2);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

// Any power-of-two complex transform, natural order in and out.
vs_status c2c(int logn, bool inv, const float2 *in, float2 *out, int batch,
              hipStream_t s) {
  if (logn <= kMaxLdsLog) return launch_c2c_lds(logn, inv, in, out, batch, s);
  int log1, log2;
  four_step_split(logn, &log1, &log2);
  const size_t bytes = (static_cast<size_t>(1) << logn) * sizeof(float2) * batch;
  DeviceBuffer tmp;
  VS_TRY(tmp.alloc(bytes, s));
  float2 *t = tmp.as<float2>();
  if (!inv) {
    // cols (+twiddle) -> rows -> transpose
    VS_TRY(launch_cols(logn, false, in, t, batch, s));
    VS_TRY(launch_c2c_lds(log2, false, t, t, batch << log1, s));
    return launch_transpose(log1, log2, t, out, batch, s);
  }
  // Inverse of the same factorisation: undo the transpose, rows, cols.
  VS_TRY(launch_transpose(log2, log1, in, t, batch, s));
  VS_TRY(launch_c2c_lds(log2, true, t, t, batch << log1, s));
  return launch_cols(logn, true, t, out, batch, s);
}


vs_status conv_four_step(int logm, const float *x, int xlen, int64_t xs, int batch,
                         const float2 *H, float *y, int64_t ys, int ylen, float2 *z,
                         hipStream_t s) {
  int log1, log2;
  four_step_split(logm, &log1, &log2);
  VS_REQUIRE(log1 >= 1 && log1 <= 10 && log2 >= 5 && log2 <= kMaxLdsLog,
             "four-step convolution: bad split of 2^%d", logm);
  vs_status st;
  const float2 *tw1 = twiddles(log1, &st);
  if (!tw1) return st;
  const float2 *tw2 = twiddles(log2, &st);
  if (!tw2) return st;
  const float2 *tws = split_twiddles(logm, &st);
  if (!tws) return st;
  const int sh = split_shift(logm);
  const int npairs = (batch + 1) / 2;
  switch (log1) {
#define VS_CASE(L) \
  case L: launch_pack_t<L>(x, xlen, xs, batch, z, log2, tw1, tws, sh, s); break;
    VS_CASE(1) VS_CASE(2) VS_CASE(3) VS_CASE(4) VS_CASE(5) VS_CASE(6) VS_CASE(7)
    VS_CASE(8) VS_CASE(9) VS_CASE(10)
#undef VS_CASE
  }
  switch (log2) {
#define VS_CASE(L) \
  case L: launch_rows_conv_t<L>(z, H, log1, npairs, tw2, s); break;
    VS_CASE(5) VS_CASE(6) VS_CASE(7) VS_CASE(8) VS_CASE(9) VS_CASE(10) VS_CASE(11)
    VS_CASE(12) VS_CASE(13) VS_CASE(14)
#undef VS_CASE
  }
  const float scale = 1.0f / static_cast<float>(1LL << logm);
  switch (log1) {
#define VS_CASE(L) \
  case L: launch_unpack_t<L>(z, log2, batch, y, ys, ylen, scale, tw1, tws, sh, s); break;
    VS_CASE(1) VS_CASE(2) VS_CASE(3) VS_CASE(4) VS_CASE(5) VS_CASE(6) VS_CASE(7)
    VS_CASE(8) VS_CASE(9) VS_CASE(10)
#undef VS_CASE
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // namespace fft
}  // namespace vs

using namespace vs;

extern "C" {

vs_status vs_fft_c2c(const float *in, float *out, int n, int batch, int inverse,
                     vs_stream_t stream) {
  const int logn = fft::ilog2_exact(n);
  VS_REQUIRE(in && out, "vs_fft_c2c: null pointer");
  VS_REQUIRE(logn >= 1 && logn <= fft::kMaxLog,
             "vs_fft_c2c: n = %d must be a power of two in [2, 2^24]", n);
  VS_REQUIRE(batch >= 0, "vs_fft_c2c: negative batch");
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_fft_c2c(in + b0 * 2 * n, out + b0 * 2 * n, n, nb, inverse, stream);
    });
  return fft::c2c(logn, inverse != 0, reinterpret_cast<const float2 *>(in),
                  reinterpret_cast<float2 *>(out), batch,
                  static_cast<hipStream_t>(stream));
}

vs_status vs_fft_r2c(const float *in, float *out, int n, int batch,
                     vs_stream_t stream) {
  const int logn = fft::ilog2_exact(n);
  VS_REQUIRE(in && out, "vs_fft_r2c: null pointer");
  VS_REQUIRE(logn >= 2 && logn <= fft::kMaxLog + 1,
             "vs_fft_r2c: n = %d must be a power of two in [4, 2^25]", n);
  if (batch <= 0) return VS_OK;
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_fft_r2c(in + b0 * n, out + b0 * (n + 2), n, nb, stream);
    });
  auto s = static_cast<hipStream_t>(stream);
  const int logh = logn - 1, h = n / 2;
  DeviceBuffer z;
  VS_TRY(z.alloc(static_cast<size_t>(h) * batch * sizeof(float2), s));
  VS_TRY(fft::c2c(logh, false, reinterpret_cast<const float2 *>(in), z.as<float2>(),
                  batch, s));
  vs_status st;
  const float2 *tw = fft::twiddles(logn, &st);
  if (!tw) return st;
  const long long work = static_cast<long long>(batch) * (h / 2 + 1);
  hipLaunchKernelGGL(fft::r2c_post_kernel, dim3(elementwise_grid(work, 256)), dim3(256),
                     0, s, z.as<float2>(), reinterpret_cast<float2 *>(out), logh,
                     batch, tw);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_fft_c2r(const float *in, float *out, int n, int batch,
                     vs_stream_t stream) {
  const int logn = fft::ilog2_exact(n);
  VS_REQUIRE(in && out, "vs_fft_c2r: null pointer");
  VS_REQUIRE(logn >= 2 && logn <= fft::kMaxLog + 1,
             "vs_fft_c2r: n = %d must be a power of two in [4, 2^25]", n);
  if (batch <= 0) return VS_OK;
  if (batch > kMaxGridY)
    return batch_chunks(batch, [&](long long b0, int nb) {
      return vs_fft_c2r(in + b0 * (n + 2), out + b0 * n, n, nb, stream);
    });
  auto s = static_cast<hipStream_t>(stream);
  const int logh = logn - 1, h = n / 2;
  DeviceBuffer z;
  VS_TRY(z.alloc(static_cast<size_t>(h) * batch * sizeof(float2), s));
  vs_status st;
  const float2 *tw = fft::twiddles(logn, &st);
  if (!tw) return st;
  const long long work = static_cast<long long>(batch) * h;
  hipLaunchKernelGGL(fft::c2r_pre_kernel, dim3(elementwise_grid(work, 256)), dim3(256),
                     0, s, reinterpret_cast<const float2 *>(in), z.as<float2>(), logh,
                     batch, tw);
  VS_HIP(hipGetLastError());
  return fft::c2c(logh, true, z.as<float2>(), reinterpret_cast<float2 *>(out), batch, s);
}

}  // extern "C"
