// matrix.h (reference src/matrix.c:255-343).  The GPU path stages host
// operands through the library stream; device operands are used in place.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/matrix.h"

#include "csrc/api/dispatch.h"
#include "csrc/ref/ref.h"
#include "simd/gpu.h"

using vs::Staged;

namespace {
// Work below which a simd = 1 call on host operands stays on the host
// (a GPU round trip is 14-18 us; the host loops run 4-16 floats per cycle).
constexpr size_t kSmallElems = vs::api::kHostAlways;  // add / sub: host operands stay on the host
constexpr size_t kSmallMacs = 3 << 19;  // multiply: 96^3 takes 12 us on the host (4 x 16 register blocks), 27 us through the GPU; 128^3 29 us on both

void elementwise(int simd, int op, const char *what, const float *m1,
                 const float *m2, size_t w, size_t h, float *res) {
  if (!m1 || !m2 || !res || w == 0 || h == 0)
    vs::fatal("%s: invalid arguments", what);
  const size_t n = w * h;
  if (simd && vs::api::host_small(n, kSmallElems, {m1, m2, res})) {
    if (op == VS_OP_ADD) vs::host::matrix_add(m1, m2, w, h, res);
    else vs::host::matrix_sub(m1, m2, w, h, res);
    return;
  }
  if (!vs::api::use_gpu_simd(simd, what)) {
    if (op == VS_OP_ADD) vs::ref::matrix_add(m1, m2, w, h, res);
    else vs::ref::matrix_sub(m1, m2, w, h, res);
    return;
  }
  vs::api::run_sync(what, [&](hipStream_t s) {
    Staged o(res, n * 4, Staged::kOut, s);
    Staged a(m1, n * 4, Staged::kIn, s), b(m2, n * 4, Staged::kIn, s);
    VS_TRY(o.status());
    VS_TRY(a.status());
    VS_TRY(b.status());
    VS_TRY(vs_binary(op, a.dev<float>(), b.dev<float>(), o.dev<float>(), n, s));
    return o.finish();
  });
}
}  // namespace

extern "C" {

void matrix_add(int simd, const float *m1, const float *m2, size_t w,
                size_t h, float *res) {
  elementwise(simd, VS_OP_ADD, "matrix_add", m1, m2, w, h, res);
}

void matrix_sub(int simd, const float *m1, const float *m2, size_t w,
                size_t h, float *res) {
  elementwise(simd, VS_OP_SUB, "matrix_sub", m1, m2, w, h, res);
}

void matrix_multiply(int simd, const float *m1, const float *m2, size_t w1,
                     size_t h1, size_t w2, size_t h2, float *res) {
  if (w1 != h2 || !m1 || !m2 || !res || !w1 || !h1 || !w2)
    vs::fatal("matrix_multiply: invalid arguments (w1=%zu h1=%zu w2=%zu h2=%zu)",
              w1, h1, w2, h2);
  if (simd && vs::api::host_small(w1 * h1 * w2, kSmallMacs, {m1, m2, res})) {
    vs::host::matrix_multiply(m1, m2, w1, h1, w2, res);
    return;
  }
  if (!vs::api::use_gpu_simd(simd, "matrix_multiply")) {
    vs::ref::matrix_multiply(m1, m2, w1, h1, w2, res);
    return;
  }
  vs::api::run_sync("matrix_multiply", [&](hipStream_t s) {
    Staged c(res, h1 * w2 * 4, Staged::kOut, s);
    Staged a(m1, h1 * w1 * 4, Staged::kInReread, s);
    Staged b(m2, h2 * w2 * 4, Staged::kInReread, s);
    VS_TRY(c.status());
    VS_TRY(a.status());
    VS_TRY(b.status());
    VS_TRY(vs_sgemm(0, 0, vs::api::checked_int("matrix_multiply", h1), vs::api::checked_int("matrix_multiply", w2),
                    vs::api::checked_int("matrix_multiply", w1), 1.f, a.dev<float>(), w1,
                    b.dev<float>(), w2, 0.f, c.dev<float>(), w2, s));
    return c.finish();
  });
}

void matrix_multiply_transposed(int simd, const float *m1, const float *m2,
                                size_t w1, size_t h1, size_t w2, size_t h2,
                                float *res) {
  if (w1 != w2 || !m1 || !m2 || !res || !w1 || !h1 || !h2)
    vs::fatal("matrix_multiply_transposed: invalid arguments "
              "(w1=%zu h1=%zu w2=%zu h2=%zu)", w1, h1, w2, h2);
  if (simd && vs::api::host_small(w1 * h1 * h2, kSmallMacs, {m1, m2, res})) {
    vs::host::matrix_multiply_transposed(m1, m2, w1, h1, h2, res);
    return;
  }
  if (!vs::api::use_gpu_simd(simd, "matrix_multiply_transposed")) {
    vs::ref::matrix_multiply_transposed(m1, m2, w1, h1, h2, res);
    return;
  }
  vs::api::run_sync("matrix_multiply_transposed", [&](hipStream_t s) {
    Staged c(res, h1 * h2 * 4, Staged::kOut, s);
    Staged a(m1, h1 * w1 * 4, Staged::kInReread, s);
    Staged b(m2, h2 * w2 * 4, Staged::kInReread, s);
    VS_TRY(c.status());
    VS_TRY(a.status());
    VS_TRY(b.status());
    VS_TRY(vs_sgemm(0, 1, vs::api::checked_int("matrix_multiply", h1), vs::api::checked_int("matrix_multiply", h2),
                    vs::api::checked_int("matrix_multiply", w1), 1.f, a.dev<float>(), w1,
                    b.dev<float>(), w2, 0.f, c.dev<float>(), h2, s));
    return c.finish();
  });
}

}  // extern "C"
