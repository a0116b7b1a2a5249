// Elementwise CDNA4 kernels: dtype conversions, real/complex arithmetic,
// fills, reversed copies and transcendental math.  These are HBM-bound; every kernel moves 4 elements per lane per
// iteration with one vector load/store per operand (16 B for fp32) when the
// pointers allow it, one vector per lane (grid-stride only past 2^20 blocks), and
// falls back to a scalar body for unaligned operands.
//
// Reference counterparts: inc/simd/arithmetic.h:43-191 (scalar semantics),
// :211-830 (AVX bodies), src/memory.c:93-183, src/matrix.c:170-198,
// inc/simd/mathfun.h:105-140.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "csrc/kernels/device.h"
#include "csrc/runtime/runtime.h"
#include "simd/device_math.h"
#include "simd/gpu.h"

namespace vs {
namespace {

using dev::Vec;
constexpr unsigned kBlock = 256;

inline bool aligned_to(const void *p, size_t a) {
  return (reinterpret_cast<uintptr_t>(p) % a) == 0;
}

// VELES_STREAM_NT=0 turns the non-temporal path of the streaming kernels off
// (A/B measurements).
inline bool stream_nt() {
  static const bool on = [] {
    const char *e = std::getenv("VELES_STREAM_NT");
    return !(e && e[0] == '0');
  }();
  return on;
}

// ------------------------------------------------------------ conversions
template <class In, class Out>
struct Convert;

template <>
struct Convert<int16_t, float> {
  __device__ float operator()(int16_t v) const { return static_cast<float>(v); }
};
template <>
struct Convert<int32_t, float> {
  __device__ float operator()(int32_t v) const { return static_cast<float>(v); }
};
template <>
struct Convert<float, int32_t> {
  // v_cvt_i32_f32: truncation toward zero, saturating, NaN -> 0.
  __device__ int32_t operator()(float v) const { return __float2int_rz(v); }
};
template <>
struct Convert<float, int16_t> {
  __device__ int16_t operator()(float v) const {
    int32_t t = __float2int_rz(v);
    t = t < -32768 ? -32768 : (t > 32767 ? 32767 : t);
    return static_cast<int16_t>(t);
  }
};
template <>
struct Convert<int32_t, int16_t> {
  __device__ int16_t operator()(int32_t v) const {
    v = v < -32768 ? -32768 : (v > 32767 ? 32767 : v);
    return static_cast<int16_t>(v);
  }
};
template <>
struct Convert<int16_t, int32_t> {
  __device__ int32_t operator()(int16_t v) const { return v; }
};
template <>
struct Convert<uint16_t, float> {
  // v_cvt_f32_f16: exact for normals, subnormals, +-inf and NaN.
  __device__ float operator()(uint16_t v) const {
    return static_cast<float>(__builtin_bit_cast(_Float16, v));
  }
};
template <>
struct Convert<uint8_t, float> {
  __device__ float operator()(uint8_t v) const { return static_cast<float>(v); }
};
template <>
struct Convert<float, float> {
  __device__ float operator()(float v) const { return v; }
};

// NT: arrays too large for the caches to matter stream through with
// non-temporal loads and stores (kStreamBytes).
constexpr size_t kStreamBytes = static_cast<size_t>(64) << 20;

template <class In, class Out, class F, int V, bool NT>
__global__ __launch_bounds__(kBlock) void map1_kernel(
    const In *__restrict__ in, Out *__restrict__ out, size_t n, F f) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const size_t nv = n / V;
  for (size_t i = tid; i < nv; i += stride) {
    const Vec<In, V> a = dev::load_vec<NT>(reinterpret_cast<const Vec<In, V> *>(in) + i);
    Vec<Out, V> r;
#pragma unroll
    for (int j = 0; j < V; j++) r.v[j] = f(a.v[j]);
    dev::store_vec<NT>(reinterpret_cast<Vec<Out, V> *>(out) + i, r);
  }
  for (size_t i = nv * V + tid; i < n; i += stride) out[i] = f(in[i]);
}

template <class In, class Out, class F>
vs_status launch_map1(const In *in, Out *out, size_t n, F f,
                      hipStream_t stream) {
  if (n == 0) return VS_OK;
  constexpr int V = 4;
  const bool vec = aligned_to(in, sizeof(In) * V) && aligned_to(out, sizeof(Out) * V);
  const unsigned grid = elementwise_grid(vec ? (n + V - 1) / V : n, kBlock);
  if (vec && n * (sizeof(In) + sizeof(Out)) >= kStreamBytes && stream_nt())
    hipLaunchKernelGGL((map1_kernel<In, Out, F, V, true>), dim3(grid), dim3(kBlock),
                       0, stream, in, out, n, f);
  else if (vec)
    hipLaunchKernelGGL((map1_kernel<In, Out, F, V, false>), dim3(grid), dim3(kBlock),
                       0, stream, in, out, n, f);
  else
    hipLaunchKernelGGL((map1_kernel<In, Out, F, 1, false>), dim3(grid), dim3(kBlock),
                       0, stream, in, out, n, f);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

template <class A, class B, class Out, class F, int V, bool NT>
__global__ __launch_bounds__(kBlock) void map2_kernel(
    const A *__restrict__ a, const B *__restrict__ b, Out *__restrict__ out,
    size_t n, F f) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const size_t nv = n / V;
  for (size_t i = tid; i < nv; i += stride) {
    const Vec<A, V> x = dev::load_vec<NT>(reinterpret_cast<const Vec<A, V> *>(a) + i);
    const Vec<B, V> y = dev::load_vec<NT>(reinterpret_cast<const Vec<B, V> *>(b) + i);
    Vec<Out, V> r;
#pragma unroll
    for (int j = 0; j < V; j++) r.v[j] = f(x.v[j], y.v[j]);
    dev::store_vec<NT>(reinterpret_cast<Vec<Out, V> *>(out) + i, r);
  }
  for (size_t i = nv * V + tid; i < n; i += stride) out[i] = f(a[i], b[i]);
}

template <class A, class B, class Out, class F>
vs_status launch_map2(const A *a, const B *b, Out *out, size_t n, F f,
                      hipStream_t stream) {
  if (n == 0) return VS_OK;
  constexpr int V = 4;
  const bool vec = aligned_to(a, sizeof(A) * V) && aligned_to(b, sizeof(B) * V) &&
                   aligned_to(out, sizeof(Out) * V);
  const unsigned grid = elementwise_grid(vec ? (n + V - 1) / V : n, kBlock);
  if (vec && n * (sizeof(A) + sizeof(B) + sizeof(Out)) >= kStreamBytes && stream_nt())
    hipLaunchKernelGGL((map2_kernel<A, B, Out, F, V, true>), dim3(grid), dim3(kBlock),
                       0, stream, a, b, out, n, f);
  else if (vec)
    hipLaunchKernelGGL((map2_kernel<A, B, Out, F, V, false>), dim3(grid), dim3(kBlock),
                       0, stream, a, b, out, n, f);
  else
    hipLaunchKernelGGL((map2_kernel<A, B, Out, F, 1, false>), dim3(grid), dim3(kBlock),
                       0, stream, a, b, out, n, f);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

struct AddOp {
  __device__ float operator()(float x, float y) const { return x + y; }
};
struct SubOp {
  __device__ float operator()(float x, float y) const { return x - y; }
};
struct MulOp {
  __device__ float operator()(float x, float y) const { return x * y; }
};
struct Int16MulOp {
  __device__ int32_t operator()(int16_t x, int16_t y) const {
    return static_cast<int32_t>(x) * static_cast<int32_t>(y);
  }
};
struct AffineOp {
  float scale, shift;
  __device__ float operator()(float x) const { return x * scale + shift; }
};
struct ScaleOp {
  float scale;
  __device__ float operator()(float x) const { return x * scale; }
};
struct ShiftOp {
  float shift;
  __device__ float operator()(float x) const { return x + shift; }
};
struct SaxpyOp {
  float a;
  __device__ float operator()(float x, float y) const { return fmaf(a, x, y); }
};

// The element functions are the public device-callable ones
// (include/simd/device_math.h), so user kernels compose exactly what the
// array kernels run.
template <int FN>
struct MathOp {
  __device__ float operator()(float x) const {
    if constexpr (FN == VS_FN_SIN) return simd_sin_ps(x);
    if constexpr (FN == VS_FN_COS) return simd_cos_ps(x);
    if constexpr (FN == VS_FN_LOG) return simd_log_ps(x);
    if constexpr (FN == VS_FN_SQRT) return simd_sqrt_ps(x);
    return simd_exp_ps(x);
  }
};
// x^y evaluated in double and rounded once: OCML powf was measured at up
// to 5 ulp (15.65^4.2); the double pow keeps every result within 1 ulp.
// FP64 VALU runs at half the FP32 rate, which this HBM-bound map never
// reaches (12 bytes per element).
struct PowOp {
  __device__ float operator()(float x, float y) const {
    return simd_pow_ps(x, y);
  }
};

// float4 access, non-temporal when `nt` (uniform): see kStreamBytes.
__device__ __forceinline__ float4 ld4(const float4 *p, bool nt) {
  typedef float native4 __attribute__((ext_vector_type(4)));
  if (nt) {
    const native4 r = __builtin_nontemporal_load(reinterpret_cast<const native4 *>(p));
    return make_float4(r.x, r.y, r.z, r.w);
  }
  return *p;
}
__device__ __forceinline__ void st4(float4 *p, float4 v, bool nt) {
  typedef float native4 __attribute__((ext_vector_type(4)));
  if (nt) {
    const native4 r = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(r, reinterpret_cast<native4 *>(p));
  } else {
    *p = v;
  }
}

// sin and cos of the same argument: one shared range reduction per element
// (OCML sincosf), two 16-byte stores per lane.
__global__ __launch_bounds__(kBlock) void sincos_kernel(const float *__restrict__ x,
                                                        float *__restrict__ s,
                                                        float *__restrict__ c, size_t n,
                                                        bool nt) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const size_t nv = n / 4;
  for (size_t i = tid; i < nv; i += stride) {
    const float4 v = ld4(reinterpret_cast<const float4 *>(x) + i, nt);
    float4 sv, cv;
    simd_sincos_ps4(v, &sv, &cv);
    st4(reinterpret_cast<float4 *>(s) + i, sv, nt);
    st4(reinterpret_cast<float4 *>(c) + i, cv, nt);
  }
  for (size_t i = 4 * nv + tid; i < n; i += stride) simd_sincos_ps(x[i], s + i, c + i);
}

__global__ __launch_bounds__(kBlock) void sincos_scalar_kernel(const float *__restrict__ x,
                                                               float *__restrict__ s,
                                                               float *__restrict__ c, size_t n) {
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  for (size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x; i < n; i += stride)
    simd_sincos_ps(x[i], s + i, c + i);
}

// ------------------------------------------------------- complex kernels
// Two interleaved complex numbers per lane (one float4).
template <bool CONJ, int V>
__global__ __launch_bounds__(kBlock) void cmul_kernel(
    const float2 *__restrict__ a, const float2 *__restrict__ b,
    float2 *__restrict__ out, size_t n, bool nt) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const size_t nv = n / V;
  for (size_t i = tid; i < nv; i += stride) {
    Vec<float2, V> x, y, r;
    if constexpr (V == 2) {
      x = __builtin_bit_cast(Vec<float2, V>, ld4(reinterpret_cast<const float4 *>(a) + i, nt));
      y = __builtin_bit_cast(Vec<float2, V>, ld4(reinterpret_cast<const float4 *>(b) + i, nt));
    } else {
      x = reinterpret_cast<const Vec<float2, V> *>(a)[i];
      y = reinterpret_cast<const Vec<float2, V> *>(b)[i];
    }
#pragma unroll
    for (int j = 0; j < V; j++) {
      const float yi = CONJ ? -y.v[j].y : y.v[j].y;
      r.v[j].x = x.v[j].x * y.v[j].x - x.v[j].y * yi;
      r.v[j].y = x.v[j].x * yi + y.v[j].x * x.v[j].y;
    }
    if constexpr (V == 2)
      st4(reinterpret_cast<float4 *>(out) + i, __builtin_bit_cast(float4, r), nt);
    else
      reinterpret_cast<Vec<float2, V> *>(out)[i] = r;
  }
  for (size_t i = nv * V + tid; i < n; i += stride) {
    const float yi = CONJ ? -b[i].y : b[i].y;
    float2 r;
    r.x = a[i].x * b[i].x - a[i].y * yi;
    r.y = a[i].x * yi + b[i].x * a[i].y;
    out[i] = r;
  }
}

// VEC: two complex numbers (one float4) per lane, both pointers 16-byte
// aligned; the scalar tail / unaligned path flips every odd float.
template <bool VEC>
__global__ __launch_bounds__(kBlock) void conj_kernel(const float *__restrict__ a,
                                                      float *__restrict__ out,
                                                      size_t n, bool nt) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  size_t done = 0;
  if (VEC) {
    const size_t n4 = n / 4;
    for (size_t i = tid; i < n4; i += stride) {
      float4 v = ld4(reinterpret_cast<const float4 *>(a) + i, nt);
      v.y = -v.y;
      v.w = -v.w;
      st4(reinterpret_cast<float4 *>(out) + i, v, nt);
    }
    done = n4 * 4;
  }
  for (size_t i = done + tid; i < n; i += stride) out[i] = (i & 1) ? -a[i] : a[i];
}

__global__ __launch_bounds__(kBlock) void fill_kernel(float *__restrict__ p,
                                                      float v, size_t n) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  const bool vec = (reinterpret_cast<uintptr_t>(p) & 15) == 0;
  size_t done = 0;
  if (vec) {
    const size_t n4 = n / 4;
    const float4 f = make_float4(v, v, v, v);
    for (size_t i = tid; i < n4; i += stride) reinterpret_cast<float4 *>(p)[i] = f;
    done = n4 * 4;
  }
  for (size_t i = done + tid; i < n; i += stride) p[i] = v;
}

template <bool PAIRS, bool VEC = false>
__global__ __launch_bounds__(kBlock) void reverse_kernel(
    const float *__restrict__ src, float *__restrict__ dst, size_t n, bool nt) {
  const size_t tid = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  const size_t stride = static_cast<size_t>(gridDim.x) * blockDim.x;
  if (PAIRS) {
    const size_t np = n / 2;
    const float2 *s = reinterpret_cast<const float2 *>(src);
    float2 *d = reinterpret_cast<float2 *>(dst);
    for (size_t i = tid; i < np; i += stride) d[i] = s[np - 1 - i];
  } else if (VEC) {
    // dst 16-byte aligned and src + n 16-byte aligned: dst float4 i is the
    // reversed float4 of src ending at n - 4 i; the last n % 4 outputs come
    // from src[0 .. n % 4) (3.6 -> ~5.8 TB/s at 2^26, tools/bench_memops.py)
    const size_t n4 = n / 4;
    const float4 *s4 = reinterpret_cast<const float4 *>(src + n) - 1;
    for (size_t i = tid; i < n4; i += stride) {
      const float4 v = ld4(s4 - i, nt);
      st4(reinterpret_cast<float4 *>(dst) + i, make_float4(v.w, v.z, v.y, v.x), nt);
    }
    for (size_t i = 4 * n4 + tid; i < n; i += stride) dst[i] = src[n - 1 - i];
  } else {
    for (size_t i = tid; i < n; i += stride) dst[i] = src[n - 1 - i];
  }
}

}  // namespace
}  // namespace vs

using namespace vs;

extern "C" {

vs_status vs_convert(const void *src, int st, void *dst, int dt, size_t n,
                     vs_stream_t stream) {
  auto s = static_cast<hipStream_t>(stream);
  VS_REQUIRE(src && dst, "vs_convert: null pointer");
#define VS_CONV(ST, SD, DT, DD)                                               \
  if (st == SD && dt == DD)                                                   \
    return launch_map1(static_cast<const ST *>(src), static_cast<DT *>(dst), \
                       n, Convert<ST, DT>{}, s);
  VS_CONV(int16_t, VS_I16, float, VS_F32)
  VS_CONV(int32_t, VS_I32, float, VS_F32)
  VS_CONV(float, VS_F32, int32_t, VS_I32)
  VS_CONV(float, VS_F32, int16_t, VS_I16)
  VS_CONV(int32_t, VS_I32, int16_t, VS_I16)
  VS_CONV(int16_t, VS_I16, int32_t, VS_I32)
  VS_CONV(uint16_t, VS_F16, float, VS_F32)
  VS_CONV(uint8_t, VS_U8, float, VS_F32)
  VS_CONV(float, VS_F32, float, VS_F32)
#undef VS_CONV
  set_error("vs_convert: unsupported conversion %d -> %d", st, dt);
  return VS_ERR_UNSUPPORTED;
}

vs_status vs_binary(int op, const float *a, const float *b, float *out,
                    size_t n, vs_stream_t stream) {
  auto s = static_cast<hipStream_t>(stream);
  VS_REQUIRE(a && b && out, "vs_binary: null pointer");
  switch (op) {
    case VS_OP_ADD:
      return launch_map2(a, b, out, n, AddOp{}, s);
    case VS_OP_SUB:
      return launch_map2(a, b, out, n, SubOp{}, s);
    case VS_OP_MUL:
      return launch_map2(a, b, out, n, MulOp{}, s);
  }
  set_error("vs_binary: unknown op %d", op);
  return VS_ERR_INVALID;
}

vs_status vs_complex_multiply(const float *a, const float *b, float *out,
                              size_t n, int conjugate_b, vs_stream_t stream) {
  auto s = static_cast<hipStream_t>(stream);
  VS_REQUIRE(a && b && out, "vs_complex_multiply: null pointer");
  if (n == 0) return VS_OK;
  auto ca = reinterpret_cast<const float2 *>(a);
  auto cb = reinterpret_cast<const float2 *>(b);
  auto co = reinterpret_cast<float2 *>(out);
  const bool vec = aligned_to(a, 16) && aligned_to(b, 16) && aligned_to(out, 16);
  const unsigned grid = elementwise_grid(vec ? n / 2 + 1 : n, kBlock);
  const bool nt = n * 24 >= kStreamBytes && stream_nt();
  if (conjugate_b) {
    if (vec)
      hipLaunchKernelGGL((cmul_kernel<true, 2>), dim3(grid), dim3(kBlock), 0, s, ca, cb, co, n, nt);
    else
      hipLaunchKernelGGL((cmul_kernel<true, 1>), dim3(grid), dim3(kBlock), 0, s, ca, cb, co, n, nt);
  } else {
    if (vec)
      hipLaunchKernelGGL((cmul_kernel<false, 2>), dim3(grid), dim3(kBlock), 0, s, ca, cb, co, n, nt);
    else
      hipLaunchKernelGGL((cmul_kernel<false, 1>), dim3(grid), dim3(kBlock), 0, s, ca, cb, co, n, nt);
  }
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_complex_conjugate(const float *a, float *out, size_t n,
                               vs_stream_t stream) {
  VS_REQUIRE(a && out, "vs_complex_conjugate: null pointer");
  if (n == 0) return VS_OK;
  // Reference semantics (arithmetic.h:162-168): pairs (2i, 2i+1) with
  // 2i+1 < n are conjugated; an odd trailing float is not written.
  const size_t even = n & ~static_cast<size_t>(1);
  if (even == 0) return VS_OK;
  // one float4 per lane (3.6 -> ~5.8 TB/s at 2^26, tools/bench_memops.py)
  if (aligned_to(a, 16) && aligned_to(out, 16))
    hipLaunchKernelGGL(conj_kernel<true>, dim3(elementwise_grid(even / 4 + 1, kBlock)),
                       dim3(kBlock), 0, static_cast<hipStream_t>(stream), a, out, even,
                       even * 8 >= kStreamBytes && stream_nt());
  else
    hipLaunchKernelGGL(conj_kernel<false>, dim3(elementwise_grid(even, kBlock)),
                       dim3(kBlock), 0, static_cast<hipStream_t>(stream), a, out, even, false);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_affine(const float *x, float scale, float shift, float *out,
                    size_t n, vs_stream_t stream) {
  auto s = static_cast<hipStream_t>(stream);
  VS_REQUIRE(x && out, "vs_affine: null pointer");
  // Keep the exact reference arithmetic for the pure scale / pure shift
  // cases (no fused multiply-add rounding difference).
  if (shift == 0.f) return launch_map1(x, out, n, ScaleOp{scale}, s);
  if (scale == 1.f) return launch_map1(x, out, n, ShiftOp{shift}, s);
  return launch_map1(x, out, n, AffineOp{scale, shift}, s);
}

vs_status vs_saxpy(float a, const float *x, float *y, size_t n,
                   vs_stream_t stream) {
  VS_REQUIRE(x && y, "vs_saxpy: null pointer");
  return launch_map2(x, static_cast<const float *>(y), y, n, SaxpyOp{a},
                     static_cast<hipStream_t>(stream));
}

vs_status vs_fill(float *dst, float value, size_t n, vs_stream_t stream) {
  VS_REQUIRE(dst, "vs_fill: null pointer");
  if (n == 0) return VS_OK;
  hipLaunchKernelGGL(fill_kernel, dim3(elementwise_grid(n / 4 + 1, kBlock)),
                     dim3(kBlock), 0, static_cast<hipStream_t>(stream), dst,
                     value, n);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_reverse(const float *src, float *dst, size_t n, int pairs,
                     vs_stream_t stream) {
  VS_REQUIRE(src && dst, "vs_reverse: null pointer");
  VS_REQUIRE(src != dst, "vs_reverse: in-place reversal is not supported");
  if (n == 0) return VS_OK;
  auto s = static_cast<hipStream_t>(stream);
  if (pairs)
    hipLaunchKernelGGL(reverse_kernel<true>, dim3(elementwise_grid(n / 2, kBlock)),
                       dim3(kBlock), 0, s, src, dst, n, false);
  else if (aligned_to(dst, 16) && aligned_to(src + n, 16))
    hipLaunchKernelGGL((reverse_kernel<false, true>), dim3(elementwise_grid(n / 4 + 1, kBlock)),
                       dim3(kBlock), 0, s, src, dst, n, n * 8 >= kStreamBytes && stream_nt());
  else
    hipLaunchKernelGGL(reverse_kernel<false>, dim3(elementwise_grid(n, kBlock)),
                       dim3(kBlock), 0, s, src, dst, n, false);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

vs_status vs_int16_multiply(const int16_t *a, const int16_t *b, int32_t *out,
                            size_t n, vs_stream_t stream) {
  VS_REQUIRE(a && b && out, "vs_int16_multiply: null pointer");
  return launch_map2(a, b, out, n, Int16MulOp{}, static_cast<hipStream_t>(stream));
}

vs_status vs_math(int fn, const float *x, float *y, size_t n,
                  vs_stream_t stream) {
  auto s = static_cast<hipStream_t>(stream);
  VS_REQUIRE(x && y, "vs_math: null pointer");
  switch (fn) {
    case VS_FN_SIN:
      return launch_map1(x, y, n, MathOp<VS_FN_SIN>{}, s);
    case VS_FN_COS:
      return launch_map1(x, y, n, MathOp<VS_FN_COS>{}, s);
    case VS_FN_LOG:
      return launch_map1(x, y, n, MathOp<VS_FN_LOG>{}, s);
    case VS_FN_EXP:
      return launch_map1(x, y, n, MathOp<VS_FN_EXP>{}, s);
    case VS_FN_SQRT:
      return launch_map1(x, y, n, MathOp<VS_FN_SQRT>{}, s);
  }
  set_error("vs_math: unknown function %d", fn);
  return VS_ERR_INVALID;
}

vs_status vs_pow(const float *x, const float *y, float *out, size_t n, vs_stream_t stream) {
  VS_REQUIRE(x && y && out, "vs_pow: null pointer");
  return launch_map2(x, y, out, n, PowOp{}, static_cast<hipStream_t>(stream));
}

vs_status vs_sincos(const float *x, float *s, float *c, size_t n, vs_stream_t stream) {
  VS_REQUIRE(x && s && c, "vs_sincos: null pointer");
  if (n == 0) return VS_OK;
  auto st = static_cast<hipStream_t>(stream);
  const auto al = [](const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (al(x) && al(s) && al(c))
    hipLaunchKernelGGL(sincos_kernel, dim3(elementwise_grid((n + 3) / 4, kBlock)), dim3(kBlock),
                       0, st, x, s, c, n, n * 12 >= kStreamBytes && stream_nt());
  else
    hipLaunchKernelGGL(sincos_scalar_kernel, dim3(elementwise_grid(n, kBlock)), dim3(kBlock), 0,
                       st, x, s, c, n);
  VS_HIP(hipGetLastError());
  return VS_OK;
}

}  // extern "C"
