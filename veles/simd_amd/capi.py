"""numpy access to the source-compatible C API (``include/simd/*.h``).

These wrappers call exactly the exported C symbols a C/C++ user of the
reference would call (``matrix_multiply``, ``convolve_fft``, ...), with host
numpy buffers, so the Python test-suite exercises the same entry points as
the native C test binary.  ``simd`` keeps its reference meaning: 1 = the
accelerated (GPU) path, 0 = the host reference.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_vp, _i, _sz, _f = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_float

# Enums (include/simd/*.h)
WAVELET_TYPE_DAUBECHIES, WAVELET_TYPE_COIFLET, WAVELET_TYPE_SYMLET = 0, 1, 2
EXTENSION_TYPE_PERIODIC, EXTENSION_TYPE_MIRROR = 0, 1
EXTENSION_TYPE_CONSTANT, EXTENSION_TYPE_ZERO = 2, 3
kExtremumTypeMaximum, kExtremumTypeMinimum, kExtremumTypeBoth = 1, 2, 3
kConvolutionAlgorithmBruteForce, kConvolutionAlgorithmFFT = 0, 1
kConvolutionAlgorithmOverlapSave = 2


class ConvolutionOverlapSaveHandle(ctypes.Structure):
    _fields_ = [("fft_plan", _vp), ("fft_inverse_plan", _vp),
                ("fft_boiler_plate", _vp), ("H", _vp), ("x_length", _sz),
                ("h_length", _sz), ("L", _vp), ("reverse", _i)]


class ConvolutionFFTHandle(ctypes.Structure):
    _fields_ = [("fft_plan", _vp), ("fft_inverse_plan", _vp), ("M", _vp),
                ("x_length", _i), ("h_length", _i), ("inputs", _vp),
                ("reverse", _i)]


class _HandleUnion(ctypes.Union):
    _fields_ = [("fft", ConvolutionFFTHandle), ("os", ConvolutionOverlapSaveHandle)]


class ConvolutionHandle(ctypes.Structure):
    _fields_ = [("algorithm", _i), ("x_length", _i), ("h_length", _i),
                ("handle", _HandleUnion)]


class ExtremumPoint(ctypes.Structure):
    _fields_ = [("position", _i), ("value", _f)]


_SIG = {
    "matrix_add": (None, [_i, _vp, _vp, _sz, _sz, _vp]),
    "matrix_sub": (None, [_i, _vp, _vp, _sz, _sz, _vp]),
    "matrix_multiply": (None, [_i, _vp, _vp, _sz, _sz, _sz, _sz, _vp]),
    "matrix_multiply_transposed": (None, [_i, _vp, _vp, _sz, _sz, _sz, _sz, _vp]),
    "sin_psv": (None, [_i, _vp, _sz, _vp]),
    "cos_psv": (None, [_i, _vp, _sz, _vp]),
    "log_psv": (None, [_i, _vp, _sz, _vp]),
    "exp_psv": (None, [_i, _vp, _sz, _vp]),
    "sqrt_psv": (None, [_i, _vp, _sz, _vp]),
    "sincos_psv": (None, [_i, _vp, _sz, _vp, _vp]),
    "pow_psv": (None, [_i, _vp, _vp, _sz, _vp]),
    "normalize2D": (None, [_i, _vp, _i, _i, _i, _vp, _i]),
    "minmax2D": (None, [_i, _vp, _i, _i, _i, _vp, _vp]),
    "normalize2D_minmax": (None, [_i, ctypes.c_uint8, ctypes.c_uint8, _vp, _i,
                                  _i, _i, _vp, _i]),
    "minmax1D": (None, [_i, _vp, _i, _vp, _vp]),
    "detect_peaks": (None, [_i, _vp, _sz, _i, _vp, _vp]),
    "convolve_simd": (None, [_i, _vp, _sz, _vp, _sz, _vp]),
    "cross_correlate_simd": (None, [_i, _vp, _sz, _vp, _sz, _vp]),
    "convolve_fft_initialize": (ConvolutionFFTHandle, [_sz, _sz]),
    "convolve_fft": (None, [ConvolutionFFTHandle, _vp, _vp, _vp]),
    "convolve_fft_finalize": (None, [ConvolutionFFTHandle]),
    "cross_correlate_fft_initialize": (ConvolutionFFTHandle, [_sz, _sz]),
    "cross_correlate_fft": (None, [ConvolutionFFTHandle, _vp, _vp, _vp]),
    "cross_correlate_fft_finalize": (None, [ConvolutionFFTHandle]),
    "convolve_overlap_save_initialize": (ConvolutionOverlapSaveHandle, [_sz, _sz]),
    "convolve_overlap_save": (None, [ConvolutionOverlapSaveHandle, _vp, _vp, _vp]),
    "convolve_overlap_save_finalize": (None, [ConvolutionOverlapSaveHandle]),
    "cross_correlate_overlap_save_initialize": (ConvolutionOverlapSaveHandle,
                                                [_sz, _sz]),
    "cross_correlate_overlap_save": (None, [ConvolutionOverlapSaveHandle, _vp,
                                            _vp, _vp]),
    "cross_correlate_overlap_save_finalize": (None, [ConvolutionOverlapSaveHandle]),
    "convolve_initialize": (ConvolutionHandle, [_sz, _sz]),
    "convolve": (None, [ConvolutionHandle, _vp, _vp, _vp]),
    "convolve_finalize": (None, [ConvolutionHandle]),
    "cross_correlate_initialize": (ConvolutionHandle, [_sz, _sz]),
    "cross_correlate": (None, [ConvolutionHandle, _vp, _vp, _vp]),
    "cross_correlate_finalize": (None, [ConvolutionHandle]),
    "wavelet_validate_order": (_i, [_i, _i]),
    "wavelet_apply": (None, [_i, _i, _i, _vp, _sz, _vp, _vp]),
    "wavelet_apply_na": (None, [_i, _i, _i, _vp, _sz, _vp, _vp]),
    "stationary_wavelet_apply": (None, [_i, _i, _i, _i, _vp, _sz, _vp, _vp]),
    "stationary_wavelet_apply_na": (None, [_i, _i, _i, _i, _vp, _sz, _vp, _vp]),
    "sum_elements": (_f, [_vp, _sz]),
    "sum_elements_na": (_f, [_vp, _sz]),
    "next_highest_power_of_2": (_i, [_i]),
    "free": (None, [_vp]),
}

_CONV_NAMES = {"int16_to_float", "float_to_int16", "int32_to_float",
               "float_to_int32", "int16_to_int32", "int32_to_int16",
               "float16_to_float"}
for _n in list(_CONV_NAMES):
    _SIG[_n] = (None, [_vp, _sz, _vp])
    _SIG[_n + "_na"] = (None, [_vp, _sz, _vp])
for _n in ("real_multiply_array", "real_multiply_array_na"):
    _SIG[_n] = (None, [_vp, _vp, _sz, _vp])
for _n in ("real_multiply_scalar", "real_multiply_scalar_na", "add_to_all",
           "add_to_all_na"):
    _SIG[_n] = (None, [_vp, _sz, _f, _vp])
for _n in ("complex_conjugate", "complex_conjugate_na"):
    _SIG[_n] = (None, [_vp, _sz, _vp])
for _n in ("real_multiply", "complex_multiply", "complex_multiply_conjugate",
           "int16_multiply", "real_multiply_na", "complex_multiply_na",
           "complex_multiply_conjugate_na"):
    _SIG[_n] = (None, [_vp, _vp, _vp])

_bound: dict = {}


def fn(name: str):
    """The bound C function ``name`` (libc ``free`` is resolved too)."""
    f = _bound.get(name)
    if f is None:
        lib = _lib.lib()
        f = getattr(ctypes.CDLL(None), name) if name == "free" else getattr(lib, name)
        res, args = _SIG[name]
        f.restype = res
        f.argtypes = args
        _bound[name] = f
    return f


def p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


class PinnedArray:
    """A float32 numpy array in page-locked memory from vs_host_alloc: the
    host API reads and writes such operands by DMA (or in place) instead of
    through the pageable staging copies.  Keep the object alive while the
    array is in use; close() (or the context manager) frees the memory."""

    def __init__(self, n: int):
        self._ptr = _lib.lib().vs_host_alloc(n * 4)
        if not self._ptr:
            raise MemoryError(f"vs_host_alloc({n * 4}) failed")
        buf = (ctypes.c_float * n).from_address(self._ptr)
        self.array = np.frombuffer(buf, dtype=np.float32, count=n)

    def close(self):
        if self._ptr:
            self.array = None
            _lib.lib().vs_host_free(self._ptr)
            self._ptr = None

    def __enter__(self):
        return self.array

    def __exit__(self, *exc):
        self.close()


# ------------------------------------------------------------------ helpers
def matrix_multiply(simd, m1, m2, w1, h1, w2, h2):
    m1, m2 = f32(m1), f32(m2)
    res = np.empty(h1 * w2, np.float32)
    fn("matrix_multiply")(simd, p(m1), p(m2), w1, h1, w2, h2, p(res))
    return res


def matrix_multiply_transposed(simd, m1, m2, w1, h1, w2, h2):
    m1, m2 = f32(m1), f32(m2)
    res = np.empty(h1 * h2, np.float32)
    fn("matrix_multiply_transposed")(simd, p(m1), p(m2), w1, h1, w2, h2, p(res))
    return res


def matrix_add(simd, m1, m2, w, h):
    m1, m2 = f32(m1), f32(m2)
    res = np.empty(w * h, np.float32)
    fn("matrix_add")(simd, p(m1), p(m2), w, h, p(res))
    return res


def matrix_sub(simd, m1, m2, w, h):
    m1, m2 = f32(m1), f32(m2)
    res = np.empty(w * h, np.float32)
    fn("matrix_sub")(simd, p(m1), p(m2), w, h, p(res))
    return res


def psv(name, simd, x):
    x = f32(x)
    res = np.empty_like(x)
    fn(name)(simd, p(x), x.size, p(res))
    return res


def sincos_psv(simd, x):
    x = f32(x)
    s, c = np.empty_like(x), np.empty_like(x)
    fn("sincos_psv")(simd, p(x), x.size, p(s), p(c))
    return s, c


def pow_psv(simd, x, y):
    x, y = f32(x), f32(y)
    res = np.empty_like(x)
    fn("pow_psv")(simd, p(x), p(y), x.size, p(res))
    return res


def convolve_simd(simd, x, h, correlate=False):
    x, h = f32(x), f32(h)
    res = np.empty(x.size + h.size - 1, np.float32)
    fn("cross_correlate_simd" if correlate else "convolve_simd")(
        simd, p(x), x.size, p(h), h.size, p(res))
    return res


def run_handle(prefix, x, h):
    """``<prefix>_initialize`` -> ``<prefix>`` -> ``<prefix>_finalize``."""
    x, h = f32(x), f32(h)
    handle = fn(prefix + "_initialize")(x.size, h.size)
    res = np.empty(x.size + h.size - 1, np.float32)
    fn(prefix)(handle, p(x), p(h), p(res))
    fn(prefix + "_finalize")(handle)
    return res, handle


def detect_peaks(simd, x, kind):
    x = f32(x)
    out = ctypes.POINTER(ExtremumPoint)()
    count = ctypes.c_size_t(0)
    fn("detect_peaks")(simd, p(x), x.size, kind, ctypes.byref(out),
                       ctypes.byref(count))
    pts = [(out[i].position, out[i].value) for i in range(count.value)]
    if out:
        fn("free")(ctypes.cast(out, _vp))
    return pts


def wavelet_apply(type_, order, ext, src, na=False):
    src = f32(src)
    hi = np.empty(src.size // 2, np.float32)
    lo = np.empty(src.size // 2, np.float32)
    fn("wavelet_apply_na" if na else "wavelet_apply")(
        type_, order, ext, p(src), src.size, p(hi), p(lo))
    return hi, lo


def stationary_wavelet_apply(type_, order, level, ext, src, na=False):
    src = f32(src)
    hi = np.empty(src.size, np.float32)
    lo = np.empty(src.size, np.float32)
    fn("stationary_wavelet_apply_na" if na else "stationary_wavelet_apply")(
        type_, order, level, ext, p(src), src.size, p(hi), p(lo))
    return hi, lo
