/*! @file arithmetic.h
 *  @brief Conversions, real/complex arithmetic and reductions.
 *
 *  Source-compatible with reference inc/simd/arithmetic.h.  In the
 *  reference these are static inline SSE/AVX/NEON bodies; here they are
 *  exported library functions with two execution paths:
 *   - array functions (conversions, *_array, complex_conjugate,
 *     real_multiply_scalar, sum_elements, add_to_all) run as HIP kernels when
 *     an operand lives in device memory, and as host loops otherwise: on
 *     host arrays one pass of the CPU costs less than the copy into pinned
 *     memory the GPU path starts with (real_multiply_array over 1 Mi floats:
 *     108 us on the host, 490 us through the GPU).  VELES_GPU_MIN_ELEMS=n
 *     sends host arrays of n elements or more to the GPU all the same;
 *   - the fixed-width "register" helpers (real_multiply, complex_multiply,
 *     complex_multiply_conjugate: FLOAT_STEP floats; int16_multiply:
 *     INT16MUL_STEP elements) are host helpers with the reference AVX2
 *     semantics; their array-sized GPU counterparts are in simd/gpu.h.
 *  The *_na functions are the scalar reference semantics (reference
 *  arithmetic.h:43-191) and always run on the host.
 *
 *  Semantics follow the scalar reference, not its SIMD quirks:
 *  int16 inputs are sign-extended in order; float -> int conversion
 *  truncates toward zero; narrowing to int16 saturates (the tests only use
 *  in-range values, where this equals the reference cast).
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_ARITHMETIC_H_
#define VELES_SIMD_ARITHMETIC_H_

#include <stddef.h>
#include <stdint.h>
#include <simd/attributes.h>
#include <simd/common.h>
#include <simd/instruction_set.h>
#include <simd/memory.h>

/// Floats processed by one call of the fixed-width helpers (as AVX).
#define FLOAT_STEP 8
#define FLOAT_STEP_LOG2 3
/// int16 elements processed by one int16_multiply() call (as AVX2).
#define INT16MUL_STEP 16
#define INT16MUL_STEP_LOG2 4

SIMD_API_BEGIN

typedef union {
  uint32_t i;
  float f;
} FloatUint32;

/* ---- scalar reference (host) ------------------------------------------ */
void int16_to_float_na(const int16_t *data, size_t length, float *res)
    NOTNULL(1, 3);
void float_to_int16_na(const float *data, size_t length, int16_t *res)
    NOTNULL(1, 3);
void int32_to_float_na(const int32_t *data, size_t length, float *res)
    NOTNULL(1, 3);
void float_to_int32_na(const float *data, size_t length, int32_t *res)
    NOTNULL(1, 3);
void int32_to_int16_na(const int32_t *data, size_t length, int16_t *res)
    NOTNULL(1, 3);
void int16_to_int32_na(const int16_t *data, size_t length, int32_t *res)
    NOTNULL(1, 3);
void float16_to_float_na(const uint16_t *data, size_t length, float *res)
    NOTNULL(1, 3);
void real_multiply_na(const float *a, const float *b, float *res)
    NOTNULL(1, 2, 3);
void real_multiply_array_na(const float *a, const float *b, size_t length,
                            float *res) NOTNULL(1, 2, 4);
void complex_multiply_na(const float *a, const float *b, float *res)
    NOTNULL(1, 2, 3);
void complex_multiply_conjugate_na(const float *a, const float *b,
                                   float *res) NOTNULL(1, 2, 3);
void complex_conjugate_na(const float *array, size_t length, float *res)
    NOTNULL(1, 3);
void real_multiply_scalar_na(const float *array, size_t length, float value,
                             float *res) NOTNULL(1, 4);
float sum_elements_na(const float *input, size_t length) NOTNULL(1);
void add_to_all_na(float *input, size_t length, float value, float *output)
    NOTNULL(1, 4);

/* ---- accelerated ------------------------------------------------------- */
/// res[i] = (int32)a[i] * b[i], i < INT16MUL_STEP.
void int16_multiply(const int16_t *a, const int16_t *b, int32_t *res)
    NOTNULL(1, 2, 3);
void int16_to_float(const int16_t *data, size_t length, float *res)
    NOTNULL(1, 3);
void float_to_int16(const float *data, size_t length, int16_t *res)
    NOTNULL(1, 3);
void int32_to_float(const int32_t *data, size_t length, float *res)
    NOTNULL(1, 3);
void float_to_int32(const float *data, size_t length, int32_t *res)
    NOTNULL(1, 3);
void int16_to_int32(const int16_t *data, size_t length, int32_t *res)
    NOTNULL(1, 3);
void int32_to_int16(const int32_t *data, size_t length, int16_t *res)
    NOTNULL(1, 3);
/// IEEE-754 binary16 (as raw uint16) -> float, subnormals/inf/NaN exact.
void float16_to_float(const uint16_t *data, size_t length, float *res)
    NOTNULL(1, 3);
/// res[i] = a[i] * b[i], i < FLOAT_STEP.
void real_multiply(const float *a, const float *b, float *res)
    NOTNULL(1, 2, 3);
void real_multiply_array(const float *a, const float *b, size_t length,
                         float *res) NOTNULL(1, 2, 4);
/// Interleaved complex product of FLOAT_STEP floats (FLOAT_STEP/2 numbers).
void complex_multiply(const float *a, const float *b, float *res)
    NOTNULL(1, 2, 3);
/// a * conj(b) over FLOAT_STEP floats.
void complex_multiply_conjugate(const float *a, const float *b, float *res)
    NOTNULL(1, 2, 3);
void complex_conjugate(const float *array, size_t length, float *res)
    NOTNULL(1, 3);
void real_multiply_scalar(const float *array, size_t length, float value,
                          float *res) NOTNULL(1, 4);
float sum_elements(const float *input, size_t length) NOTNULL(1);
void add_to_all(float *input, size_t length, float value, float *output)
    NOTNULL(1, 4);

/// Smallest power of two >= value (reference arithmetic.h:1227-1235).
int next_highest_power_of_2(int value);

SIMD_API_END

#endif  // VELES_SIMD_ARITHMETIC_H_
