// Host-side FFT plans: twiddle tables and the launchers the convolution
// kernels share.  Replaces the reference's external FFTF dependency
// (reference src/convolve.c:131-143, fftf_init / fftf_calc / fftf_destroy).
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#pragma once

#include <hip/hip_runtime.h>

#include "csrc/runtime/runtime.h"

namespace vs {
namespace fft {

constexpr int kMaxLdsLog = 14;   // largest single-workgroup (LDS) transform
constexpr int kMaxLog = 24;      // largest transform (four-step)

// exp(-2 pi i m / 2^logn), m < 2^logn, on the current device (cached; the
// first request per (device, size) allocates and uploads synchronously).
const float2 *twiddles(int logn, vs_status *st);

// Split tables for exp(-2 pi i a / 2^logn), a < 2^logn, as
// hi[a >> s] * lo[a & (2^s - 1)] with s = ceil(logn / 2): `lo` has 2^s
// entries, `hi` 2^(logn - s).  Returned as one buffer: lo then hi.
const float2 *split_twiddles(int logn, vs_status *st);
inline int split_shift(int logn) { return (logn + 1) / 2; }

// Four-step geometry for 2^logn = N1 x N2 (N1 = 2^log1 <= 1024 columns
// transformed first, N2 = 2^log2 <= 16384 contiguous rows).
inline void four_step_split(int logn, int *log1, int *log2) {
  int l2 = logn - 4;
  if (l2 > kMaxLdsLog) l2 = kMaxLdsLog;
  if (logn - l2 > 10) l2 = logn - 10;
  *log2 = l2;
  *log1 = logn - l2;
}

// Batched contiguous complex FFT with n = 2^logn <= 2^kMaxLdsLog points.
vs_status launch_c2c_lds(int logn, bool inverse, const float2 *in, float2 *out,
                         int batch, hipStream_t s);
// Column pass of the four-step transform on `batch` signals of N1 x N2:
// forward: FFT_N1 over columns, then * W_N^(n2 k1), out[k1][n2];
// inverse: * conj W_N^(n2 k1), then IFFT_N1 over columns.
vs_status launch_cols(int logn, bool inverse, const float2 *in, float2 *out,
                      int batch, hipStream_t s);
// Whole-signal FFT convolution of `batch` real signals (packed in pairs into
// z: (batch + 1) / 2 x 2^logm complex scratch) with the four-step-layout
// filter spectrum H (cols + rows forward of the padded filter): three fused
// passes, outputs scaled by 2^-logm straight to y (ylen per row).
vs_status conv_four_step(int logm, const float *x, int xlen, int64_t xs, int batch,
                         const float2 *H, float *y, int64_t ys, int ylen, float2 *z,
                         hipStream_t s);
// out[sig][k1 + N1 k2] = in[sig][k1][k2]  (N1 x N2 -> natural order).
vs_status launch_transpose(int log1, int log2, const float2 *in, float2 *out,
                           int batch, hipStream_t s);

int ilog2_exact(long long n);  // -1 if n is not a power of two

}  // namespace fft
}  // namespace vs
