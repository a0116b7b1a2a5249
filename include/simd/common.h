/*! @file common.h
 *  @brief C linkage / symbol visibility wrappers for the public API.
 *
 *  Same contract as the reference's SIMD_API_BEGIN/END
 *  (reference inc/simd/common.h:34-51): every public function has C
 *  linkage and default visibility, so the library can be hidden-by-default.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_COMMON_H_
#define VELES_SIMD_COMMON_H_

#ifdef __cplusplus
#define SIMD_API_BEGIN \
  extern "C" {         \
  _Pragma("GCC visibility push(default)")
#define SIMD_API_END             \
  _Pragma("GCC visibility pop") \
  }
#else
#define SIMD_API_BEGIN _Pragma("GCC visibility push(default)")
#define SIMD_API_END _Pragma("GCC visibility pop")
#endif

#endif  // VELES_SIMD_COMMON_H_
