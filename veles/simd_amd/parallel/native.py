"""Python face of the native multi-GPU layer (csrc/dist/dist.cpp,
include/simd/dist.h): one process drives every local MI355X, RCCL over xGMI
(``backend="rccl"``) or stream-ordered peer copies (``backend="local"``, which
also lets several ranks share one GPU -- the single-GPU test double).

This is the counterpart of the torch.distributed helpers in this package for
C-API users (one process, many devices).
"""
from __future__ import annotations

import ctypes
from typing import Sequence

import numpy as np

from .. import _lib

BACKENDS = {"auto": 0, "rccl": 1, "local": 2}
_BACKEND_NAMES = {v: k for k, v in BACKENDS.items()}
EXTENSIONS = {"periodic": 0, "mirror": 1, "constant": 2, "zero": 3}
WAVELETS = {"daubechies": 0, "coiflet": 1, "symlet": 2}


def shard(n: int, nranks: int, rank: int) -> tuple[int, int]:
    """(begin, count) of rank's contiguous shard (first n % nranks get +1)."""
    b, c = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.lib().vs_dist_shard(n, nranks, rank, ctypes.byref(b), ctypes.byref(c))
    return b.value, c.value


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _ptr(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _ptr_array(ptrs: Sequence[int]):
    return (ctypes.c_void_p * len(ptrs))(*ptrs)


class DeviceGroup:
    """A communicator over ``nranks`` ranks (devices default to r mod count)."""

    def __init__(self, nranks: int, devices: Sequence[int] | None = None,
                 backend: str = "auto", timeout_ms: int | None = None):
        lib = _lib.lib()
        h = ctypes.c_void_p()
        devs = None
        if devices is not None:
            assert len(devices) == nranks
            devs = (ctypes.c_int * nranks)(*devices)
        _lib.check(lib.vs_dist_create(nranks, devs, BACKENDS[backend], ctypes.byref(h)),
                   "vs_dist_create")
        self._h = h
        if timeout_ms is not None:
            _lib.check(lib.vs_dist_set_timeout(h, timeout_ms), "vs_dist_set_timeout")

    # ---------------------------------------------------------------- info
    @property
    def size(self) -> int:
        return _lib.lib().vs_dist_size(self._h)

    @property
    def backend(self) -> str:
        return _BACKEND_NAMES[_lib.lib().vs_dist_backend_of(self._h)]

    def device(self, rank: int) -> int:
        return _lib.lib().vs_dist_device(self._h, rank)

    def stream(self, rank: int) -> int:
        return _lib.lib().vs_dist_stream(self._h, rank) or 0

    def synchronize(self) -> None:
        _lib.check(_lib.lib().vs_dist_synchronize(self._h), "vs_dist_synchronize")

    def close(self) -> None:
        if self._h:
            _lib.lib().vs_dist_destroy(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------ collectives on per-rank tensors
    # Tensors are torch CUDA tensors, one per rank on that rank's device; the
    # call enqueues on the ranks' library streams and synchronises.
    def broadcast(self, tensors, root: int = 0) -> None:
        p = _ptr_array([t.data_ptr() for t in tensors])
        nbytes = tensors[0].numel() * tensors[0].element_size()
        self._sync_inputs(tensors)
        _lib.check(_lib.lib().vs_dist_broadcast(self._h, p, nbytes, root), "vs_dist_broadcast")
        self.synchronize()

    def all_gather(self, send, recv) -> None:
        s = _ptr_array([t.data_ptr() for t in send])
        r = _ptr_array([t.data_ptr() for t in recv])
        nbytes = send[0].numel() * send[0].element_size()
        self._sync_inputs(send)
        _lib.check(_lib.lib().vs_dist_all_gather(self._h, s, r, nbytes), "vs_dist_all_gather")
        self.synchronize()

    def all_reduce_sum(self, tensors) -> None:
        p = _ptr_array([t.data_ptr() for t in tensors])
        self._sync_inputs(tensors)
        _lib.check(_lib.lib().vs_dist_all_reduce_sum(self._h, p, tensors[0].numel()),
                   "vs_dist_all_reduce_sum")
        self.synchronize()

    def halo_exchange(self, src, halo, direction: int = 1, periodic: bool = False) -> None:
        s = _ptr_array([t.data_ptr() for t in src])
        hh = _ptr_array([t.data_ptr() for t in halo])
        lens = (ctypes.c_size_t * len(src))(*[t.numel() for t in src])
        self._sync_inputs(src)
        _lib.check(_lib.lib().vs_dist_halo_exchange(self._h, s, lens, hh, halo[0].numel(),
                                                    direction, int(periodic)),
                   "vs_dist_halo_exchange")
        self.synchronize()

    def sgemm_rowsplit_device(self, a_rows, b, c) -> None:
        """Device-resident row-split batched GEMM: a_rows[r] = rank r's rows
        ([batch, rows_r, k], rows_r = shard(m, size, r)), b[r] = the full
        [batch, k, n] and c[r] = a [batch, m, n] output on rank r's device;
        on return every c[r] holds the whole product (rows all-gathered)."""
        batch, _, k = a_rows[0].shape
        m, n = c[0].shape[-2], c[0].shape[-1]
        pa = _ptr_array([t.data_ptr() for t in a_rows])
        pb = _ptr_array([t.data_ptr() for t in b])
        pc = _ptr_array([t.data_ptr() for t in c])
        self._sync_inputs(list(a_rows) + list(b))
        _lib.check(_lib.lib().vs_dist_sgemm_rowsplit_device(self._h, m, n, k, pa, pb, pc,
                                                            batch),
                   "vs_dist_sgemm_rowsplit_device")
        self.synchronize()

    @staticmethod
    def _sync_inputs(tensors) -> None:
        import torch
        for d in {t.device for t in tensors}:
            torch.cuda.synchronize(d)

    # ------------------------------------------ sharded host-array entry points
    def sgemm_rowsplit(self, a, b) -> np.ndarray:
        """Batched C = A @ B with A's rows split over ranks ([batch,] m, k)."""
        a, b = _f32(a), _f32(b)
        squeeze = a.ndim == 2
        if squeeze:
            a, b = a[None], b[None]
        batch, m, k = a.shape
        n = b.shape[2]
        assert b.shape == (batch, k, n)
        c = np.empty((batch, m, n), np.float32)
        _lib.check(_lib.lib().vs_dist_sgemm_rowsplit(self._h, m, n, k, _ptr(a), _ptr(b),
                                                     _ptr(c), batch), "vs_dist_sgemm_rowsplit")
        return c[0] if squeeze else c

    def conv1d_batch(self, x, h, correlate: bool = False) -> np.ndarray:
        x, h = _f32(x), _f32(h)
        batch, xl = x.shape
        y = np.empty((batch, xl + h.size - 1), np.float32)
        _lib.check(_lib.lib().vs_dist_conv1d_batch(self._h, int(correlate), _ptr(x), xl,
                                                   _ptr(h), h.size, _ptr(y), batch),
                   "vs_dist_conv1d_batch")
        return y

    def swt_batch(self, x, wavelet: str = "daubechies", order: int = 8, levels: int = 1,
                  ext: str = "periodic") -> tuple[np.ndarray, np.ndarray]:
        """Data-parallel stationary wavelet transform of the rows of x
        [batch, len]: (hi [batch, levels, len], lo [batch, len])."""
        x = _f32(x)
        batch, n = x.shape
        hi = np.empty((batch, levels, n), np.float32)
        lo = np.empty((batch, n), np.float32)
        _lib.check(_lib.lib().vs_dist_swt_batch(self._h, WAVELETS[wavelet], order, levels,
                                                EXTENSIONS[ext], _ptr(x), n, batch, _ptr(hi),
                                                _ptr(lo)), "vs_dist_swt_batch")
        return hi, lo

    def swt_batch_device(self, x, hi, lo, wavelet: str = "daubechies", order: int = 8,
                         levels: int = 1, ext: str = "periodic") -> None:
        """Device-resident data-parallel SWT: x[r] [rows_r, len], hi[r]
        [rows_r, levels, len], lo[r] [rows_r, len] are rank r's tensors on its
        device; enqueued on the ranks' streams and synchronised."""
        n = x[0].shape[-1]
        counts = (ctypes.c_int * len(x))(*[t.shape[0] for t in x])
        self._sync_inputs(list(x))
        _lib.check(_lib.lib().vs_dist_swt_batch_device(
            self._h, WAVELETS[wavelet], order, levels, EXTENSIONS[ext],
            _ptr_array([t.data_ptr() for t in x]), n, counts,
            _ptr_array([t.data_ptr() for t in hi]), _ptr_array([t.data_ptr() for t in lo])),
            "vs_dist_swt_batch_device")
        self.synchronize()

    def dwt_batch(self, x, wavelet: str = "daubechies", order: int = 8, levels: int = 1,
                  ext: str = "periodic") -> np.ndarray:
        """Data-parallel decimated pyramid of the rows of x [batch, len]:
        rows [hi_1 | hi_2 | ... | hi_L | lo_L]."""
        x = _f32(x)
        batch, n = x.shape
        out = np.empty((batch, n), np.float32)
        _lib.check(_lib.lib().vs_dist_dwt_batch(self._h, WAVELETS[wavelet], order, levels,
                                                EXTENSIONS[ext], _ptr(x), n, batch, _ptr(out)),
                   "vs_dist_dwt_batch")
        return out

    def sgemm_batch(self, a, b, trans_a: bool = False, trans_b: bool = False) -> np.ndarray:
        """Data-parallel batched C[i] = op(A[i]) op(B[i]), matrices sharded
        over ranks."""
        a, b = _f32(a), _f32(b)
        batch = a.shape[0]
        m, k = (a.shape[2], a.shape[1]) if trans_a else (a.shape[1], a.shape[2])
        n = b.shape[1] if trans_b else b.shape[2]
        c = np.empty((batch, m, n), np.float32)
        _lib.check(_lib.lib().vs_dist_sgemm_batch(self._h, int(trans_a), int(trans_b), m, n, k,
                                                  _ptr(a), _ptr(b), _ptr(c), batch),
                   "vs_dist_sgemm_batch")
        return c

    def conv1d_long(self, x, h, correlate: bool = False) -> np.ndarray:
        x, h = _f32(x), _f32(h)
        y = np.empty(x.size + h.size - 1, np.float32)
        _lib.check(_lib.lib().vs_dist_conv1d_long(self._h, int(correlate), _ptr(x), x.size,
                                                  _ptr(h), h.size, _ptr(y)),
                   "vs_dist_conv1d_long")
        return y

    def swt_long(self, x, wavelet: str = "daubechies", order: int = 8, levels: int = 1,
                 ext: str = "periodic") -> tuple[np.ndarray, np.ndarray]:
        """Returns (hi [levels, len], lo [len])."""
        x = _f32(x)
        hi = np.empty((levels, x.size), np.float32)
        lo = np.empty(x.size, np.float32)
        _lib.check(_lib.lib().vs_dist_swt_long(self._h, WAVELETS[wavelet], order, levels,
                                               EXTENSIONS[ext], _ptr(x), x.size, _ptr(hi),
                                               _ptr(lo)), "vs_dist_swt_long")
        return hi, lo
