/*! @file instruction_set.h
 *  @brief Accelerator selection.
 *
 *  The reference picks SSE/AVX/AVX2/NEON intrinsics here
 *  (reference inc/simd/instruction_set.h:34-66).  This library has exactly
 *  one accelerated target: AMD Instinct MI355X (gfx950, CDNA4).  There are no
 *  host intrinsics and no CPU-SIMD dual path: the "SIMD" path of every public
 *  function runs as a HIP kernel, the scalar path (simd == 0 / *_na) is the
 *  CPU reference implementation.
 *  Copyright 2026 veles.simd_amd authors. Apache-2.0.
 */
#ifndef VELES_SIMD_INSTRUCTION_SET_H_
#define VELES_SIMD_INSTRUCTION_SET_H_

/// Always defined: the accelerated path is available at compile time.  Whether
/// a GPU is present is a runtime question (vs_gpu_available(), simd/gpu.h).
#define SIMD 1
#define VELES_SIMD_TARGET_GFX950 1
/// Lane width of one hardware wavefront on CDNA4.
#define VELES_SIMD_WAVEFRONT 64

#endif  // VELES_SIMD_INSTRUCTION_SET_H_
