"""Helpers shared by the torch custom-op wrappers."""
from __future__ import annotations

import ctypes
import contextlib

import torch

from .. import _lib


def ptr(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr())


def stream_of(t: torch.Tensor) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


@contextlib.contextmanager
def on_device(t: torch.Tensor):
    """Make t's GPU the current HIP device for the native launch."""
    if t.is_cuda:
        with torch.cuda.device(t.device):
            yield
    else:
        yield


def require_gpu_tensor(t: torch.Tensor, name: str) -> None:
    """GPU tensors must run the native kernels; fail loudly if unavailable."""
    if not _lib.available():
        raise _lib.NativeLibraryMissing(
            f"{name}: native library not built; refusing a silent fallback")
    if not _lib.gpu_available():
        raise _lib.VelesError(f"{name}: native library sees no GPU")


def contiguous_f32(t: torch.Tensor, name: str) -> torch.Tensor:
    if t.dtype != torch.float32:
        raise TypeError(f"{name}: expected float32, got {t.dtype}")
    return t.contiguous()
