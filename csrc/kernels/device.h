// Device-side helpers shared by the CDNA4 kernels.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace vs {
namespace dev {

constexpr int kWave = 64;  // CDNA wavefront width

template <class T, int N>
struct alignas(sizeof(T) * N) Vec {
  T v[N];
};

// Streaming access for data touched once: non-temporal loads and stores keep
// it out of the way of what the caches could still serve (a stream of 10 %
// reads among writes ran 5.56 TB/s with plain loads, 5.79 with these).
template <bool NT, class T, int N>
__device__ __forceinline__ Vec<T, N> load_vec(const Vec<T, N> *p) {
  if constexpr (NT && N > 1) {
    typedef T native __attribute__((ext_vector_type(N)));
    const native r = __builtin_nontemporal_load(reinterpret_cast<const native *>(p));
    return __builtin_bit_cast(Vec<T, N>, r);
  } else if constexpr (NT) {
    Vec<T, N> r;
    r.v[0] = __builtin_nontemporal_load(&p->v[0]);
    return r;
  } else {
    return *p;
  }
}

template <bool NT, class T, int N>
__device__ __forceinline__ void store_vec(Vec<T, N> *p, const Vec<T, N> &x) {
  if constexpr (NT && N > 1) {
    typedef T native __attribute__((ext_vector_type(N)));
    __builtin_nontemporal_store(__builtin_bit_cast(native, x), reinterpret_cast<native *>(p));
  } else if constexpr (NT) {
    __builtin_nontemporal_store(x.v[0], &p->v[0]);
  } else {
    *p = x;
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fminf(v, __shfl_xor(v, off, kWave));
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

__device__ __forceinline__ int wave_isum(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Bijective XCD-aware remap of a 1D block id (8 XCDs, round-robin dispatch):
// consecutive logical tiles land on the same XCD so they share its L2
// (cdna_hip_programming.md §5.5 T1).  Speed only, never correctness.
__device__ __forceinline__ unsigned xcd_remap(unsigned bid, unsigned nblocks) {
  constexpr unsigned kXcd = 8;
  if (nblocks < kXcd) return bid;
  const unsigned q = nblocks / kXcd, r = nblocks % kXcd;
  const unsigned xcd = bid % kXcd, pos = bid / kXcd;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + pos;
}

// Output-tile coordinates of linear tile t in GROUP-row bands: consecutive
// t walk GROUP tile rows down before moving one tile column right, so the
// blocks an XCD runs together (a contiguous t range after xcd_remap) share
// ~GROUP A panels and ~(resident / GROUP) B panels in that XCD's L2 instead
// of 2 A panels and every B panel.
template <unsigned GROUP = 8>
__device__ __forceinline__ void grouped_tile(unsigned t, unsigned tiles_m,
                                             unsigned tiles_n, unsigned &tm,
                                             unsigned &tn) {
  const unsigned band = t / (GROUP * tiles_n);
  const unsigned first = band * GROUP;
  const unsigned rows = tiles_m - first < GROUP ? tiles_m - first : GROUP;
  const unsigned in = t - band * GROUP * tiles_n;
  tm = first + in % rows;
  tn = in / rows;
}

}  // namespace dev
}  // namespace vs
