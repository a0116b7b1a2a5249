/*! @file attributes.h
 *  @brief Function attribute macros of the public API.
 *
 *  Mirrors reference inc/simd/attributes.h:34-61 (INLINE, NOTNULL, MALLOC,
 *  UNUSED, WARN_UNUSED_RESULT).  NOTNULL is disabled inside the library
 *  (VELES_SIMD_IMPLEMENTATION) because the implementation validates pointers
 *  itself and reports errors instead of letting the optimiser assume them.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_ATTRIBUTES_H_
#define VELES_SIMD_ATTRIBUTES_H_

#ifndef INLINE
#define INLINE static inline __attribute__((always_inline))
#endif

#if defined(VELES_SIMD_IMPLEMENTATION) || defined(LIBSIMD_IMPLEMENTATION)
#define NOTNULL(...)
#else
#define NOTNULL(...) __attribute__((nonnull(__VA_ARGS__)))
#endif

#define MALLOC __attribute__((malloc))
#define UNUSED __attribute__((unused))
#define WARN_UNUSED_RESULT __attribute__((warn_unused_result))

#endif  // VELES_SIMD_ATTRIBUTES_H_
