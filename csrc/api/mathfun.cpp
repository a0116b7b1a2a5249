// mathfun.h (reference inc/simd/mathfun.h:142-204) and the array forms of
// the avx_mathfun.h / neon_mathfun.h element functions (sincos, pow,
// sqrt): simd != 0 runs the HIP kernels, simd == 0 libm on the host.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/mathfun.h"
#include "simd/avx_mathfun.h"
#include "simd/neon_mathfun.h"

#include "csrc/api/dispatch.h"
#include "simd/gpu.h"

namespace {
// Arrays this short run libm on the host even with simd = 1 (1.3 ns per
// element for logf against a GPU round trip of 13-16 us).
constexpr size_t kSmallElems = 8192;

void psv(int simd, int fn, const char *what, PsvStdFunc host, const float *src,
         size_t n, float *res) {
  if (!vs::api::use_gpu_simd(simd, what) || n == 0 ||
      vs::api::host_small(n, kSmallElems, {src, res})) {
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
      vs::api::host_small(n, kSmallElems, {src, s, c})) {
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
      vs::api::host_small(n, kSmallElems / 2, {x, y, res})) {
    pow_psv_novec(x, y, n, res);
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
