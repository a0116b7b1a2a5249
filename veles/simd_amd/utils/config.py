"""Runtime configuration knobs: the environment variables read by the native
library (csrc/) and the Python layer, with their defaults and meaning.

The reference is configured only at build time (autotools flags); these are the runtime equivalents.  ``KNOBS`` is the single registry:
tests/test_config.py checks that every variable the native sources read is
listed here, and ``python -m veles.simd_amd.utils.config`` prints the
effective values of the current environment."""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Knob:
    name: str
    default: str
    doc: str
    where: str  # the file that reads it

    @property
    def value(self) -> str:
        return os.environ.get(self.name, self.default)


KNOBS = [
    Knob("VELES_LOG_LEVEL", "0", "0 quiet, 1 dispatch decisions, 2 every staging step "
         "(native stderr)", "csrc/runtime/runtime.cpp"),
    Knob("VELES_DISABLE_GPU", "0", "1: behave as if no GPU were present (host reference "
         "paths)", "csrc/runtime/runtime.cpp"),
    Knob("VELES_GPU_MIN_ELEMS", "", "when set: host arrays of at least this many elements "
         "(x taps for wavelets) run on the GPU in the flag-less API; unset, streaming calls on "
         "host arrays stay on the host (1048576 applies when VELES_HOST_SMALL_SCALE=0)",
         "csrc/runtime/runtime.cpp"),
    Knob("VELES_HOST_MAX_MACS", str(3 << 18), "convolutions of host operands (direct calls and handles) "
         "below this many multiply-adds run on the host even with simd=1", "csrc/api/convolve.cpp"),
    Knob("VELES_HOST_SMALL_SCALE", "100", "percent applied to the small-call limits below which "
         "simd=1 matrix / math calls on host operands run host loops (0: always the GPU)",
         "csrc/runtime/runtime.cpp"),
    Knob("VELES_SYNC_STAGE", "0", "1: stage host operands with synchronous copies (debug)",
         "csrc/runtime/runtime.cpp"),
    Knob("VELES_STAGE_MAX_KB", "4096", "largest pageable host operand (KiB) packed into the "
         "call's pinned staging image; larger ones take a pageable copy each",
         "csrc/runtime/runtime.cpp"),
    Knob("VELES_STAGE_ARENA_MB", "16", "size of that image (pinned host + device), per thread "
         "that calls the host API", "csrc/runtime/runtime.cpp"),
    Knob("VELES_PIPELINED_MAP", "1", "0: long host calls (math functions, convolutions) stage whole arrays "
         "instead of overlapped pieces through the pinned image", "csrc/runtime/runtime.cpp"),
    Knob("VELES_ZERO_COPY", "1", "0: stage every small host operand into device memory "
         "instead of the mapped pinned arena", "csrc/runtime/runtime.cpp"),
    Knob("VELES_SGEMM_VARIANT", "-1", "force an SGEMM tile (0 / 1 / 2: 64 / 128 / 256 tiles "
         "with automatic k slicing, 3..5: whole tiles only; include/simd/gpu.h) for tuning",
         "csrc/kernels/sgemm.hip"),
    Knob("VELES_SCRATCH_CACHE_MB", "8192", "cap of the device scratch cache (freed blocks "
         "kept for reuse, per stream); above it the oldest blocks are released",
         "csrc/runtime/runtime.cpp"),
    Knob("VELES_STREAM_NT", "1", "0: plain instead of non-temporal loads / stores in the "
         "elementwise kernels on arrays past 64 MB (A/B measurements)",
         "csrc/kernels/elementwise.hip"),
    Knob("VELES_GEMM_BF16_VARIANT", "-1", "force a bf16 GEMM variant (0: 128 tiles, "
         "1: large tiles)", "csrc/kernels/gemm_bf16.hip"),
    Knob("VELES_GEMM_BF16_PACK", "-1", "force (1) or forbid (0) the bf16 operand pre-pack "
         "pass", "csrc/kernels/gemm_bf16.hip"),
    Knob("VELES_DIST_TIMEOUT_MS", "300000", "RCCL watchdog timeout of vs_dist_synchronize",
         "csrc/dist/dist.cpp"),
    Knob("VS_EW_GRID_CAP", str(1 << 20), "elementwise grid cap in workgroups (grid-stride "
         "beyond; tuning)", "csrc/runtime/runtime.cpp"),
    Knob("VELES_PROFILE_RANGES", "0", "1: roctx range around every native call made from "
         "Python (visible in rocprofv3 --marker-trace)", "veles/simd_amd/_lib.py"),
    Knob("VELES_SIMD_LIB", "", "path of an alternative libvelessimd.so (A/B runs)",
         "veles/simd_amd/_lib.py"),
]
BY_NAME = {k.name: k for k in KNOBS}


def describe() -> str:
    """Markdown table of every knob with its effective value."""
    rows = ["| variable | value | default | meaning |", "|---|---|---|---|"]
    for k in KNOBS:
        rows.append(f"| `{k.name}` | {k.value or '-'} | {k.default or '-'} | {k.doc} |")
    return "\n".join(rows)


if __name__ == "__main__":
    print(describe())
