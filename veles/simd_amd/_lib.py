"""ctypes binding of the native library ``_native/libvelessimd.so``.

The native library holds every HIP kernel (gfx950) plus the
source-compatible C API; Python never re-implements a kernel.  ``torch`` is
imported first on purpose: PyTorch-ROCm ships its own ``libamdhip64.so.7``
and loading it before our library makes the dynamic linker resolve our HIP
dependency to the same runtime instance (one HIP runtime per process, so
device pointers and streams are shared with torch).
"""
from __future__ import annotations

import ctypes
import os
import threading

try:  # noqa: SIM105 - see module docstring
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is present in every supported env
    torch = None

_HERE = os.path.dirname(os.path.abspath(__file__))
# VELES_SIMD_LIB points at an alternative build (A/B runs of two kernel
# variants in one GPU session); default is the in-tree library.
LIB_PATH = os.environ.get("VELES_SIMD_LIB") or os.path.join(
    _HERE, "_native", "libvelessimd.so")

c_float_p = ctypes.POINTER(ctypes.c_float)
_vp = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t
_f = ctypes.c_float

# name -> (restype, argtypes) for the vs_* device API (include/simd/gpu.h).
_SIGNATURES = {
    "vs_version": (ctypes.c_char_p, []),
    "vs_gpu_available": (_i, []),
    "vs_device_count": (_i, []),
    "vs_set_device": (_i, [_i]),
    "vs_get_device": (_i, []),
    "vs_last_error": (ctypes.c_char_p, []),
    "vs_is_device_pointer": (_i, [_vp]),
    "vs_stream_synchronize": (_i, [_vp]),
    "vs_compiled_arch": (_i, []),
    "vs_host_alloc": (_vp, [_sz]),
    "vs_host_free": (None, [_vp]),
    "vs_convert": (_i, [_vp, _i, _vp, _i, _sz, _vp]),
    "vs_binary": (_i, [_i, _vp, _vp, _vp, _sz, _vp]),
    "vs_complex_multiply": (_i, [_vp, _vp, _vp, _sz, _i, _vp]),
    "vs_complex_conjugate": (_i, [_vp, _vp, _sz, _vp]),
    "vs_affine": (_i, [_vp, _f, _f, _vp, _sz, _vp]),
    "vs_saxpy": (_i, [_f, _vp, _vp, _sz, _vp]),
    "vs_fill": (_i, [_vp, _f, _sz, _vp]),
    "vs_reverse": (_i, [_vp, _vp, _sz, _i, _vp]),
    "vs_int16_multiply": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "vs_math": (_i, [_i, _vp, _vp, _sz, _vp]),
    "vs_sum": (_i, [_vp, _sz, _vp, _vp]),
    "vs_minmax": (_i, [_vp, _sz, _vp, _vp]),
    "vs_minmax2d_u8": (_i, [_vp, _i, _i, _i, _vp, _vp]),
    "vs_minmax2d_u8_batched": (_i, [_vp, _i, _i64, _i, _i, _i, _vp, _vp]),
    "vs_normalize2d_u8_batched": (_i, [_vp, _i, _i64, _i, _i, _i, _vp, _i, _i, _vp, _i, _i64,
                                       _vp]),
    "vs_detect_peaks_batched": (_i, [_vp, _sz, _i64, _sz, _i, _vp, _i, _vp, _sz, _vp, _vp]),
    "vs_normalize2d_u8": (_i, [_vp, _i, _i, _i, _vp, _i, _i, _vp, _i, _vp]),
    "vs_sgemm": (_i, [_i, _i, _i, _i, _i, _f, _vp, _i64, _vp, _i64, _f, _vp,
                      _i64, _vp]),
    "vs_sgemm_strided_batched": (_i, [_i, _i, _i, _i, _i, _f, _vp, _i64, _i64,
                                      _vp, _i64, _i64, _f, _vp, _i64, _i64, _i,
                                      _vp]),
    "vs_gemm_bf16_strided_batched": (_i, [_i, _i, _i, _i, _i, _f, _vp, _i64, _i64, _vp,
                                          _i64, _i64, _f, _vp, _i64, _i64, _i, _vp]),
    "vs_gemm_bf16_variant": (_i, [_i, _i, _i, _i, _i, _i, _f, _vp, _i64, _vp, _i64, _f,
                                  _vp, _i64, _vp]),
    "vs_sgemm_bf16x3": (_i, [_i, _i, _i, _i, _i, _f, _vp, _i64, _vp, _i64, _f, _vp,
                             _i64, _i, _vp]),
    "vs_sgemm_bf16x3_strided_batched": (_i, [_i, _i, _i, _i, _i, _f, _vp, _i64, _i64,
                                             _vp, _i64, _i64, _f, _vp, _i64, _i64, _i,
                                             _vp]),
    "vs_device_math_example": (_i, [_vp, _f, _f, ctypes.c_size_t, _vp, _vp, _vp]),
    "vs_sgemm_variant": (_i, [_i, _i, _i, _i, _i, _i, _f, _vp, _i64, _vp, _i64, _f,
                              _vp, _i64, _vp]),
    "vs_sgemm_variant_batched": (_i, [_i, _i, _i, _i, _i, _i, _f, _vp, _i64, _i64, _vp, _i64,
                                      _i64, _f, _vp, _i64, _i64, _i, _vp]),
    "vs_fft_c2c": (_i, [_vp, _vp, _i, _i, _i, _vp]),
    "vs_fft_r2c": (_i, [_vp, _vp, _i, _i, _vp]),
    "vs_fft_c2r": (_i, [_vp, _vp, _i, _i, _vp]),
    "vs_conv1d": (_i, [_i, _i, _vp, _i64, _i64, _vp, _i, _i64, _vp, _i64, _i,
                       _vp]),
    "vs_conv1d_select": (_i, [_i64, _i, _i]),
    "vs_conv1d_plan_create": (_i, [_i, _i, _i64, _vp, _i, _i64, _i, ctypes.POINTER(_vp), _vp]),
    "vs_conv1d_plan_execute": (_i, [_vp, _vp, _i64, _vp, _i64, _i, _vp]),
    "vs_conv1d_plan_info": (_i, [_vp, ctypes.POINTER(_i), ctypes.POINTER(_i)]),
    "vs_conv1d_plan_destroy": (None, [_vp]),
    "vs_conv1d_os_block": (_i, [_i]),
    "vs_tune_set": (_i, [ctypes.c_char_p, _i]),
    "vs_tune_reset": (None, []),
    "vs_pow": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "vs_sincos": (_i, [_vp, _vp, _vp, _sz, _vp]),
    "vs_dwt": (_i, [_i, _i, _i, _vp, _i64, _i64, _vp, _vp, _i64, _i, _vp]),
    "vs_swt": (_i, [_i, _i, _i, _i, _vp, _i64, _i64, _vp, _vp, _i64, _i, _vp]),
    "vs_swt_multilevel": (_i, [_i, _i, _i, _i, _vp, _i64, _vp, _vp, _i, _vp]),
    "vs_swt_multilevel_packed": (_i, [_i, _i, _i, _i, _vp, _i64, _vp, _i, _vp]),
    "vs_dwt_multilevel": (_i, [_i, _i, _i, _i, _vp, _i64, _vp, _i, _vp]),
    "vs_wavelet_filter": (_i, [_i, _i, _vp]),
    "vs_detect_peaks": (_i, [_vp, _sz, _i, _vp, _vp, _sz, _vp, _vp]),
    # multi-GPU layer (include/simd/dist.h)
    "vs_dist_create": (_i, [_i, _vp, _i, ctypes.POINTER(_vp)]),
    "vs_dist_destroy": (_i, [_vp]),
    "vs_dist_size": (_i, [_vp]),
    "vs_dist_backend_of": (_i, [_vp]),
    "vs_dist_device": (_i, [_vp, _i]),
    "vs_dist_stream": (_vp, [_vp, _i]),
    "vs_dist_set_timeout": (_i, [_vp, _i]),
    "vs_dist_synchronize": (_i, [_vp]),
    "vs_dist_shard": (None, [_sz, _i, _i, ctypes.POINTER(_sz), ctypes.POINTER(_sz)]),
    "vs_dist_broadcast": (_i, [_vp, _vp, _sz, _i]),
    "vs_dist_all_gather": (_i, [_vp, _vp, _vp, _sz]),
    "vs_dist_all_reduce_sum": (_i, [_vp, _vp, _sz]),
    "vs_dist_halo_exchange": (_i, [_vp, _vp, _vp, _vp, _sz, _i, _i]),
    "vs_dist_sgemm_rowsplit": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _i]),
    "vs_dist_sgemm_rowsplit_device": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _i]),
    "vs_dist_conv1d_batch": (_i, [_vp, _i, _vp, _i, _vp, _i, _vp, _i]),
    "vs_dist_conv1d_long": (_i, [_vp, _i, _vp, _sz, _vp, _i, _vp]),
    "vs_dist_swt_batch": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp, _vp]),
    "vs_dist_swt_batch_device": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _vp, _vp, _vp]),
    "vs_dist_dwt_batch": (_i, [_vp, _i, _i, _i, _i, _vp, _i, _i, _vp]),
    "vs_dist_sgemm_batch": (_i, [_vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _i]),
    "vs_dist_swt_long": (_i, [_vp, _i, _i, _i, _i, _vp, _sz, _vp, _vp]),
}

_lock = threading.Lock()
_lib = None
_load_error: str | None = None


class VelesError(RuntimeError):
    """A native call returned a non-zero vs_status."""


class NativeLibraryMissing(VelesError):
    """The native library is not built (run ``python -m veles.simd_amd.build``)."""


def _load():
    global _lib, _load_error
    with _lock:
        if _lib is not None or _load_error is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            _load_error = f"{LIB_PATH} not found"
            return None
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:  # pragma: no cover
            _load_error = str(e)
            return None
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def lib():
    """The loaded ctypes library; raises NativeLibraryMissing if unbuilt."""
    l = _load()
    if l is None:
        raise NativeLibraryMissing(
            f"veles.simd_amd native library unavailable ({_load_error}); "
            "build it with `python -m veles.simd_amd.build`")
    return l


def available() -> bool:
    return _load() is not None


def check(status: int, what: str = "") -> None:
    if status != 0:
        msg = lib().vs_last_error().decode(errors="replace")
        raise VelesError(f"{what or 'native call'} failed (status {status}): {msg}")


_RANGES = os.environ.get("VELES_PROFILE_RANGES", "0") == "1"


def call(name: str, *args) -> None:
    """Call a vs_* function and raise VelesError on a non-zero status.
    With VELES_PROFILE_RANGES=1 each call is a roctx range named after the
    function (utils/profiling.py), so rocprofv3 --marker-trace timelines show
    which op launched which kernels."""
    fn = getattr(lib(), name)
    if _RANGES:
        from .utils.profiling import trace_range
        with trace_range(name):
            check(fn(*args), name)
        return
    check(fn(*args), name)


def gpu_available() -> bool:
    return available() and bool(lib().vs_gpu_available())
