"""Build the native library in-tree: ``python -m veles.simd_amd.build``.

Compiles every HIP kernel for gfx950 with hipcc (cross-compiles without a
GPU) plus the C++ runtime / C API into ``veles/simd_amd/_native/`` and the
native C API test binary into ``build/tests/``.
"""
from __future__ import annotations

import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build(jobs: int | None = None, target: str = "all", verbose: bool = False) -> None:
    jobs = jobs or min(16, os.cpu_count() or 4)
    env = dict(os.environ)
    env.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    cmd = ["make", "-C", REPO, f"-j{jobs}", target]
    res = subprocess.run(cmd, env=env, capture_output=not verbose, text=True)
    if res.returncode != 0:
        out = (res.stdout or "")[-6000:] + (res.stderr or "")[-6000:]
        raise RuntimeError(f"native build failed ({' '.join(cmd)}):\n{out}")


if __name__ == "__main__":
    build(verbose="-v" in sys.argv)
    print("built", os.path.join(REPO, "veles", "simd_amd", "_native",
                                "libvelessimd.so"))
