"""Per-call timing of matrix_multiply vs matrix_multiply_transposed (host API)."""
import ctypes
import statistics
import sys
import time
import numpy as np
sys.path.insert(0, ".")
from veles.simd_amd import capi
mm = capi.fn("matrix_multiply")
mmt = capi.fn("matrix_multiply_transposed")
w1, h1, w2 = 256, 300, 1000
a = np.random.rand(h1, w1).astype(np.float32)
b = np.random.rand(w1, w2).astype(np.float32)
bt = np.ascontiguousarray(b.T)
c = np.zeros((h1, w2), np.float32)
P = lambda x: x.ctypes.data_as(ctypes.c_void_p)


def t(f, *args):
    f(*args)
    ts = []
    for _ in range(50):
        t0 = time.perf_counter(); f(*args); ts.append(time.perf_counter() - t0)
    return round(statistics.median(ts) * 1e6, 1)


for rep in range(2):
    print("mm ", t(mm, 1, P(a), P(b), w1, h1, w2, w1, P(c)),
          "mmt", t(mmt, 1, P(a), P(bt), w1, h1, w1, w2, P(c)),
          "mmt(b as bt)", t(mmt, 1, P(a), P(b), w1, h1, w1, w2, P(c)), flush=True)
