"""PyTorch-ROCm custom ops (namespace ``veles::``) over the native kernels.

Each op has a fake (meta) implementation so it composes with torch.compile
and FakeTensor tracing, runs the gfx950 HIP kernel for GPU tensors (and
refuses to run if the native library is missing, instead of silently falling
back), and runs the host reference semantics for CPU tensors.
"""
from . import blas, elementwise, signal  # noqa: F401
from .blas import gemm_bf16, matmul, matmul_transposed, sgemm, sgemm_bf16x3  # noqa: F401
from .elementwise import (add, affine, binary, complex_conjugate,  # noqa: F401
                          complex_multiply, convert, cos, exp, log, math,
                          minmax, mul, normalize2d, pow, saxpy, sin, sincos, sqrt, sub,
                          sum_all)
from .signal import (Conv1dPlan, conv1d, conv1d_algorithm, correlate, detect_peaks,  # noqa: F401
                     detect_peaks_batched, dwt, fft, irfft, rfft, swt, swt_level, wavedec,
                     wavelet_filter)

__all__ = [
    "sgemm", "sgemm_bf16x3", "gemm_bf16", "matmul", "matmul_transposed", "convert", "binary", "add", "sub",
    "mul", "complex_multiply", "complex_conjugate", "affine", "saxpy", "math",
    "sin", "cos", "log", "exp", "sum_all", "minmax", "normalize2d", "conv1d",
    "correlate", "conv1d_algorithm", "Conv1dPlan", "fft", "rfft", "irfft", "dwt", "swt",
    "wavedec", "wavelet_filter", "detect_peaks", "detect_peaks_batched", "swt_level",
]
