#!/usr/bin/env python3
"""How many 256-thread workgroups the hardware keeps resident per CU, by
LDS size and VGPR allocation (diagnostic build, `make stamps`)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from veles.simd_amd import _lib  # noqa: E402

lib = _lib.lib()
lib.vs_residency_probe.restype = ctypes.c_float
lib.vs_residency_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_longlong]
spin = 200000  # shader cycles per workgroup (~0.1 ms)
blocks = 256 * 8
base = None
for vg in (0, 128, 168, 240):
    for kb in (0, 32, 64, 80, 96):
        ms = lib.vs_residency_probe(kb * 1024, vg, blocks, spin)
        print(f"VGPR>={vg:3d} LDS {kb:3d} KiB: {ms:.3f} ms for 8 waves-of-WGs per CU"
              f" -> ~{8 * 0.0833 / ms:.2f} resident per CU (if 2.4 GHz)", flush=True)
for w in (0, 1):
    arr = (ctypes.c_int * 5)()
    rc = lib.vs_conv_attrs(w, arr)
    print("attrs", ["real_conv<13,32>", "residency<240>"][w], rc, list(arr))
print("API occupancy real_conv<13,32>:", lib.vs_conv_occupancy(0))
