/*! @file memory.h
 *  @brief Aligned host allocation and float buffer utilities.
 *
 *  Source-compatible with reference inc/simd/memory.h:51-179.  Allocations
 *  are 64-byte aligned (reference src/memory.c:80) and are released with
 *  free().  Large fills / copies of device-resident buffers are executed on
 *  the GPU (see simd/gpu.h); host buffers are handled on the host, where a
 *  GPU round trip could never pay off for a memcpy-class operation.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_MEMORY_H_
#define VELES_SIMD_MEMORY_H_

#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <simd/attributes.h>
#include <simd/common.h>

SIMD_API_BEGIN

/// @brief Number of elements needed to advance ptr to the next 32-byte
/// boundary: (32 - ptr % 32) / sizeof(elem), or 0 if already aligned
/// (reference src/memory.c:42-69).
int align_complement_f32(const float *ptr) NOTNULL(1);
int align_complement_i16(const int16_t *ptr) NOTNULL(1);
int align_complement_u16(const uint16_t *ptr) NOTNULL(1);
int align_complement_i32(const int32_t *ptr) NOTNULL(1);
int align_complement_u32(const uint32_t *ptr) NOTNULL(1);

/// @brief Allocates size bytes aligned to 64 bytes; dispose with free().
void *malloc_aligned(size_t size) MALLOC;

/// @brief Allocates size bytes whose address is offset bytes past a 64-byte
/// boundary (0 <= offset < 32).  Free with free(ptr - offset).
void *malloc_aligned_offset(size_t size, int offset) MALLOC;

/// @brief Allocates length floats aligned to 64 bytes.
float *mallocf(size_t length) MALLOC;

/// @brief ptr[i] = value for i in [0, length).  Accepts host or device
/// pointers (device pointers are filled by a GPU kernel).
void memsetf(float *ptr, float value, size_t length) NOTNULL(1);

/// @brief Copies ptr into a new buffer of length 2^(floor(log2 length)+2)
/// (twice the power of two strictly greater than length), zero filled past
/// length (reference src/memory.c:125-142).  *newLength receives the length.
float *zeropadding(const float *ptr, size_t length, size_t *newLength)
    NOTNULL(1, 3) MALLOC;

/// @brief zeropadding() with additionalLength extra floats allocated at the
/// end (not counted in *newLength, left uninitialised as in the reference).
float *zeropaddingex(const float *ptr, size_t length, size_t *newLength,
                     size_t additionalLength) NOTNULL(1, 3) MALLOC;

/// @brief Reversed copy: dest[i] = src[length - 1 - i].
float *rmemcpyf(float *__restrict dest, const float *__restrict src,
                size_t length) NOTNULL(1, 2);

/// @brief Reversed copy of interleaved complex numbers (length in floats):
/// complex element i of dest is complex element n-1-i of src.
float *crmemcpyf(float *__restrict dest, const float *__restrict src,
                 size_t length) NOTNULL(1, 2);

SIMD_API_END

#endif  // VELES_SIMD_MEMORY_H_
