"""Runtime configuration knobs (environment variables read by the native
library and the Python layer).  The reference is configured only at build
time (autotools flags); these are the runtime equivalents."""
from __future__ import annotations

import os
from dataclasses import dataclass, field


@dataclass(frozen=True)
class Config:
    log_level: int = field(default_factory=lambda: int(os.environ.get("VELES_LOG_LEVEL", "0")))
    gpu_min_elems: int = field(
        default_factory=lambda: int(os.environ.get("VELES_GPU_MIN_ELEMS", str(1 << 20))))
    disable_gpu: bool = field(
        default_factory=lambda: os.environ.get("VELES_DISABLE_GPU", "0") == "1")
    sgemm_variant: int = field(
        default_factory=lambda: int(os.environ.get("VELES_SGEMM_VARIANT", "-1")))
    profile_ranges: bool = field(
        default_factory=lambda: os.environ.get("VELES_PROFILE_RANGES", "0") == "1")

    DOC = {
        "VELES_LOG_LEVEL": "0 quiet, 1 dispatch decisions, 2 verbose (native stderr)",
        "VELES_GPU_MIN_ELEMS": "host arrays at least this long run on the GPU "
                               "(flag-less arithmetic.h functions)",
        "VELES_DISABLE_GPU": "1: behave as if no GPU were present",
        "VELES_SGEMM_VARIANT": "force an SGEMM tile variant (0..4) for tuning",
        "VELES_PROFILE_RANGES": "1: emit roctx ranges around Python-level ops",
    }


config = Config()
