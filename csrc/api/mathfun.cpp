// mathfun.h (reference inc/simd/mathfun.h:142-204): simd != 0 runs the
// vs_math kernel, simd == 0 libm on the host.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/mathfun.h"

#include "csrc/api/dispatch.h"
#include "simd/gpu.h"

namespace {
void psv(int simd, int fn, const char *what, PsvStdFunc host, const float *src,
         size_t n, float *res) {
  if (!vs::api::use_gpu_simd(simd, what) || n == 0) {
    func_psv_novec(host, src, n, res);
    return;
  }
  vs::api::run_sync(what, [&](hipStream_t s) {
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
}  // extern "C"
