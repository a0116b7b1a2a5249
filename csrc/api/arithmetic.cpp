// arithmetic.h (reference inc/simd/arithmetic.h).  The *_na functions are the
// scalar semantics (reference :43-191); the accelerated array functions run
// the HIP kernels of csrc/kernels/elementwise.hip / reduce.hip when the GPU
// policy of csrc/api/dispatch.h says so.
// Copyright 2026 veles.simd_amd authors. Apache-2.0.
#include "simd/arithmetic.h"

#include <cstring>

#include "csrc/api/dispatch.h"
#include "csrc/ref/ref.h"
#include "simd/gpu.h"

using vs::Staged;
using vs::api::run_sync;
using vs::api::use_gpu_array;

namespace {

template <class In, class Out>
void gpu_convert(const char *what, const In *data, size_t n, Out *res,
                 int st, int dt) {
  run_sync(what, [&](hipStream_t s) {
    Staged out(res, n * sizeof(Out), Staged::kOut, s);
    Staged in(data, n * sizeof(In), Staged::kIn, s);
    VS_TRY(out.status());
    VS_TRY(in.status());
    VS_TRY(vs_convert(in.dev<void>(), st, out.dev<void>(), dt, n, s));
    return out.finish();
  });
}

inline int16_t sat16(int32_t v) {
  return static_cast<int16_t>(v < -32768 ? -32768 : (v > 32767 ? 32767 : v));
}

inline int32_t trunc32(float v) {
  // Matches v_cvt_i32_f32 / cvtt: truncate, saturate, NaN -> 0.
  if (v != v) return 0;
  if (v >= 2147483647.f) return 2147483647;
  if (v <= -2147483648.f) return static_cast<int32_t>(0x80000000u);
  return static_cast<int32_t>(v);
}

}  // namespace

extern "C" {

/* ------------------------------------------------------------ scalar _na */
void int16_to_float_na(const int16_t *data, size_t n, float *res) {
  for (size_t i = 0; i < n; i++) res[i] = static_cast<float>(data[i]);
}
void float_to_int16_na(const float *data, size_t n, int16_t *res) {
  for (size_t i = 0; i < n; i++) res[i] = sat16(trunc32(data[i]));
}
void int32_to_float_na(const int32_t *data, size_t n, float *res) {
  for (size_t i = 0; i < n; i++) res[i] = static_cast<float>(data[i]);
}
void float_to_int32_na(const float *data, size_t n, int32_t *res) {
  for (size_t i = 0; i < n; i++) res[i] = trunc32(data[i]);
}
void int32_to_int16_na(const int32_t *data, size_t n, int16_t *res) {
  for (size_t i = 0; i < n; i++) res[i] = sat16(data[i]);
}
void int16_to_int32_na(const int16_t *data, size_t n, int32_t *res) {
  for (size_t i = 0; i < n; i++) res[i] = data[i];
}

void float16_to_float_na(const uint16_t *data, size_t n, float *res) {
  // Bit-exact binary16 -> binary32 (reference arithmetic.h:92-127).
  for (size_t i = 0; i < n; i++) {
    const uint32_t in = data[i];
    const uint32_t sign = (in & 0x8000u) << 16;
    const uint32_t exp = in & 0x7c00u;
    uint32_t mant = in & 0x03ffu;
    uint32_t bits;
    if (exp == 0) {
      if (mant == 0) {
        bits = 0;
      } else {  // subnormal: renormalise
        int e = -1;
        do {
          e++;
          mant <<= 1;
        } while ((mant & 0x0400u) == 0);
        bits = ((127u - 15u - e) << 23) | ((mant & 0x03ffu) << 13);
      }
    } else if (exp == 0x7c00u) {
      bits = 0x7f800000u | (mant << 13);
    } else {
      bits = ((in & 0x7fffu) << 13) + 0x38000000u;
    }
    FloatUint32 u;
    u.i = bits | sign;
    res[i] = u.f;
  }
}

void real_multiply_na(const float *a, const float *b, float *res) {
  *res = *a * *b;
}
void real_multiply_array_na(const float *a, const float *b, size_t n,
                            float *res) {
  for (size_t i = 0; i < n; i++) res[i] = a[i] * b[i];
}
void complex_multiply_na(const float *a, const float *b, float *res) {
  const float re1 = a[0], im1 = a[1], re2 = b[0], im2 = b[1];
  res[0] = re1 * re2 - im1 * im2;
  res[1] = re1 * im2 + re2 * im1;
}
void complex_multiply_conjugate_na(const float *a, const float *b,
                                   float *res) {
  const float re1 = a[0], im1 = a[1], re2 = b[0], im2 = -b[1];
  res[0] = re1 * re2 - im1 * im2;
  res[1] = re1 * im2 + re2 * im1;
}
void complex_conjugate_na(const float *array, size_t n, float *res) {
  for (size_t i = 1; i < n; i += 2) {
    res[i - 1] = array[i - 1];
    res[i] = -array[i];
  }
}
void real_multiply_scalar_na(const float *array, size_t n, float value,
                             float *res) {
  for (size_t i = 0; i < n; i++) res[i] = array[i] * value;
}
float sum_elements_na(const float *input, size_t n) {
  float r = 0.f;
  for (size_t i = 0; i < n; i++) r += input[i];
  return r;
}
void add_to_all_na(float *input, size_t n, float value, float *output) {
  for (size_t i = 0; i < n; i++) output[i] = input[i] + value;
}

/* ----------------------------------------------------------- accelerated */
void int16_multiply(const int16_t *a, const int16_t *b, int32_t *res) {
  for (int i = 0; i < INT16MUL_STEP; i++)
    res[i] = static_cast<int32_t>(a[i]) * static_cast<int32_t>(b[i]);
}

#define VS_CONVERT_FN(NAME, IN, OUT, ST, DT)                     \
  void NAME(const IN *data, size_t n, OUT *res) {                \
    if (use_gpu_array(n, {data, res}))                           \
      gpu_convert(#NAME, data, n, res, ST, DT);                  \
    else                                                         \
      NAME##_na(data, n, res);                                   \
  }
VS_CONVERT_FN(int16_to_float, int16_t, float, VS_I16, VS_F32)
VS_CONVERT_FN(float_to_int16, float, int16_t, VS_F32, VS_I16)
VS_CONVERT_FN(int32_to_float, int32_t, float, VS_I32, VS_F32)
VS_CONVERT_FN(float_to_int32, float, int32_t, VS_F32, VS_I32)
VS_CONVERT_FN(int16_to_int32, int16_t, int32_t, VS_I16, VS_I32)
VS_CONVERT_FN(int32_to_int16, int32_t, int16_t, VS_I32, VS_I16)
VS_CONVERT_FN(float16_to_float, uint16_t, float, VS_F16, VS_F32)
#undef VS_CONVERT_FN

void real_multiply(const float *a, const float *b, float *res) {
  for (int i = 0; i < FLOAT_STEP; i++) res[i] = a[i] * b[i];
}

void real_multiply_array(const float *a, const float *b, size_t n,
                         float *res) {
  if (!use_gpu_array(n, {a, b, res})) return real_multiply_array_na(a, b, n, res);
  run_sync("real_multiply_array", [&](hipStream_t s) {
    Staged o(res, n * 4, Staged::kOut, s);
    Staged x(a, n * 4, Staged::kIn, s), y(b, n * 4, Staged::kIn, s);
    VS_TRY(o.status());
    VS_TRY(x.status());
    VS_TRY(y.status());
    VS_TRY(vs_binary(VS_OP_MUL, x.dev<float>(), y.dev<float>(), o.dev<float>(), n, s));
    return o.finish();
  });
}

void complex_multiply(const float *a, const float *b, float *res) {
  for (int i = 0; i < FLOAT_STEP; i += 2) complex_multiply_na(a + i, b + i, res + i);
}

void complex_multiply_conjugate(const float *a, const float *b, float *res) {
  for (int i = 0; i < FLOAT_STEP; i += 2)
    complex_multiply_conjugate_na(a + i, b + i, res + i);
}

void complex_conjugate(const float *array, size_t n, float *res) {
  if (!use_gpu_array(n, {array, res})) return complex_conjugate_na(array, n, res);
  run_sync("complex_conjugate", [&](hipStream_t s) {
    Staged o(res, n * 4, Staged::kInOut, s);  // odd tail float is preserved
    Staged x(array, n * 4, Staged::kIn, s);
    VS_TRY(o.status());
    VS_TRY(x.status());
    VS_TRY(vs_complex_conjugate(x.dev<float>(), o.dev<float>(), n, s));
    return o.finish();
  });
}

void real_multiply_scalar(const float *array, size_t n, float value,
                          float *res) {
  if (!use_gpu_array(n, {array, res}))
    return real_multiply_scalar_na(array, n, value, res);
  run_sync("real_multiply_scalar", [&](hipStream_t s) {
    Staged o(res, n * 4, Staged::kOut, s);
    Staged x(array, n * 4, Staged::kIn, s);
    VS_TRY(o.status());
    VS_TRY(x.status());
    VS_TRY(vs_affine(x.dev<float>(), value, 0.f, o.dev<float>(), n, s));
    return o.finish();
  });
}

float sum_elements(const float *input, size_t n) {
  if (!use_gpu_array(n, {input})) return vs::host::sum_elements(input, n);
  float result = 0.f;
  run_sync("sum_elements", [&](hipStream_t s) {
    Staged x(input, n * 4, Staged::kIn, s);
    Staged r(&result, sizeof(float), Staged::kOut, s);
    VS_TRY(x.status());
    VS_TRY(r.status());
    VS_TRY(vs_sum(x.dev<float>(), n, r.dev<float>(), s));
    return r.finish();
  });
  return result;
}

void add_to_all(float *input, size_t n, float value, float *output) {
  if (!use_gpu_array(n, {input, output})) return add_to_all_na(input, n, value, output);
  run_sync("add_to_all", [&](hipStream_t s) {
    Staged o(output, n * 4, Staged::kOut, s);
    Staged x(input, n * 4, Staged::kIn, s);
    VS_TRY(o.status());
    VS_TRY(x.status());
    VS_TRY(vs_affine(x.dev<float>(), 1.f, value, o.dev<float>(), n, s));
    return o.finish();
  });
}

int next_highest_power_of_2(int value) {
  value--;
  value |= value >> 1;
  value |= value >> 2;
  value |= value >> 4;
  value |= value >> 8;
  value |= value >> 16;
  return ++value;
}

}  // extern "C"
