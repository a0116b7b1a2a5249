// mathfun.h (reference inc/simd/mathfun.h:142-204) and the array forms of
// the avx_mathfun.h / neon_mathfun.h element functions (sincos, pow,
// sqrt): simd != 0 runs the HIP kernels, simd == 0 libm on the host.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/mathfun.h"
#include "simd/avx_mathfun.h"
#include "simd/neon_mathfun.h"

#include "csrc/api/dispatch.h"
#include "csrc/ref/ref.h"
#include "simd/gpu.h"

namespace {
// Arrays this short stay on the host even with simd = 1.  With glibc's vector
// math (AVX2 hosts) sin / cos / log / exp / sqrt cost 0.3 ns per element, as
// much as the GPU path's copies and transfers per element on top of its
// 13 us round trip, so the GPU only pays once its overlapped pieces do
// (2^20 elements: 303 us against 325 us); sincos costs twice that, pow
// 1.7 ns per element.  Without vector math libm runs at 1.3-4.6 ns per element.
size_t small_elems(int per_elem_cost) {  // 1: one function, 2: sincos, 8: pow
  if (!vs::host::has_vector_math()) return 8192 / static_cast<size_t>(per_elem_cost > 1 ? 2 : 1);
  return per_elem_cost == 1 ? size_t{1} << 20 : per_elem_cost == 2 ? 65536 : 8192;
}

void psv(int simd, int fn, const char *what, PsvStdFunc host, const float *src,
         size_t n, float *res) {
  if (!vs::api::use_gpu_simd(simd, what) || n == 0 ||
      vs::api::host_small(n, small_elems(1), {src, res})) {
    // simd = 1 on the host: glibc's vector math (at most 4 ulp); libm otherwise
    if (!simd || !vs::host::vector_math(fn, src, nullptr, n, res))
      func_psv_novec(host, src, n, res);
    return;
  }
  vs::api::run_sync(what, [&](hipStream_t s) {
    const vs::MapArray arrays[] = {{src, nullptr, 4}, {nullptr, res, 4}};
    vs_status piped = VS_OK;
    if (vs::pipelined_map(s, n, arrays, 2, [&](void *const *d, size_t cnt, hipStream_t st) {
          return vs_math(fn, static_cast<const float *>(d[0]), static_cast<float *>(d[1]), cnt, st);
        }, &piped))
      return piped;
    vs::Staged o(res, n * 4, vs::Staged::kOut, s);
    vs::Staged x(src, n * 4, vs::Staged::kIn, s);
    VS_TRY(o.status());
    VS_TRY(x.status());
    VS_TRY(vs_math(fn, x.dev<float>(), o.dev<float>(), n, s));
    return o.finish();
  });
}
}  // namespace

extern "C" {
void sin_psv(int simd, const float *src, size_t n, float *res) {
  psv(simd, VS_FN_SIN, "sin_psv", sinf, src, n, res);
}
void cos_psv(int simd, const float *src, size_t n, float *res) {
  psv(simd, VS_FN_COS, "cos_psv", cosf, src, n, res);
}
void log_psv(int simd, const float *src, size_t n, float *res) {
  psv(simd, VS_FN_LOG, "log_psv", logf, src, n, res);
}
void exp_psv(int simd, const float *src, size_t n, float *res) {
  psv(simd, VS_FN_EXP, "exp_psv", expf, src, n, res);
}
void sqrt_psv(int simd, const float *src, size_t n, float *res) {
  psv(simd, VS_FN_SQRT, "sqrt_psv", sqrtf, src, n, res);
}

void sincos_psv(int simd, const float *src, size_t n, float *s, float *c) {
  if (!vs::api::use_gpu_simd(simd, "sincos_psv") || n == 0 ||
      vs::api::host_small(n, small_elems(2), {src, s, c})) {
    if (!simd || !vs::host::vector_math(VS_FN_COS, src, nullptr, n, c) ||
        !vs::host::vector_math(VS_FN_SIN, src, nullptr, n, s))  // s may alias src: last
      sincos_psv_novec(src, n, s, c);
    return;
  }
  vs::api::run_sync("sincos_psv", [&](hipStream_t st) {
    const vs::MapArray arrays[] = {{src, nullptr, 4}, {nullptr, s, 4}, {nullptr, c, 4}};
    vs_status piped = VS_OK;
    if (vs::pipelined_map(st, n, arrays, 3, [&](void *const *d, size_t cnt, hipStream_t q) {
          return vs_sincos(static_cast<const float *>(d[0]), static_cast<float *>(d[1]),
                           static_cast<float *>(d[2]), cnt, q);
        }, &piped))
      return piped;
    vs::Staged os(s, n * 4, vs::Staged::kOut, st);
    vs::Staged oc(c, n * 4, vs::Staged::kOut, st);
    vs::Staged x(src, n * 4, vs::Staged::kIn, st);
    VS_TRY(os.status());
    VS_TRY(oc.status());
    VS_TRY(x.status());
    VS_TRY(vs_sincos(x.dev<float>(), os.dev<float>(), oc.dev<float>(), n, st));
    VS_TRY(os.finish());
    return oc.finish();
  });
}

void pow_psv(int simd, const float *x, const float *y, size_t n, float *res) {
  if (!vs::api::use_gpu_simd(simd, "pow_psv") || n == 0 ||
      vs::api::host_small(n, small_elems(8), {x, y, res})) {
    if (!simd || !vs::host::vector_math(-1, x, y, n, res)) pow_psv_novec(x, y, n, res);
    return;
  }
  vs::api::run_sync("pow_psv", [&](hipStream_t st) {
    const vs::MapArray arrays[] = {{x, nullptr, 4}, {y, nullptr, 4}, {nullptr, res, 4}};
    vs_status piped = VS_OK;
    if (vs::pipelined_map(st, n, arrays, 3, [&](void *const *d, size_t cnt, hipStream_t q) {
          return vs_pow(static_cast<const float *>(d[0]), static_cast<const float *>(d[1]),
                        static_cast<float *>(d[2]), cnt, q);
        }, &piped))
      return piped;
    vs::Staged o(res, n * 4, vs::Staged::kOut, st);
    vs::Staged a(x, n * 4, vs::Staged::kIn, st);
    vs::Staged b(y, n * 4, vs::Staged::kIn, st);
    VS_TRY(o.status());
    VS_TRY(a.status());
    VS_TRY(b.status());
    VS_TRY(vs_pow(a.dev<float>(), b.dev<float>(), o.dev<float>(), n, st));
    return o.finish();
  });
}
}  // extern "C"
