"""Profiler ranges.  On ROCm, torch.cuda.nvtx maps to roctx, so these ranges
show up in `rocprofv3 --marker-trace` timelines next to the kernel trace.
Enabled by VELES_PROFILE_RANGES=1 (no-ops otherwise, zero cost)."""
from __future__ import annotations

import contextlib
import os

import torch

_ENABLED = os.environ.get("VELES_PROFILE_RANGES", "0") == "1"


def range_push(name: str) -> None:
    if _ENABLED and torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)


def range_pop() -> None:
    if _ENABLED and torch.cuda.is_available():
        torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def trace_range(name: str):
    range_push(name)
    try:
        yield
    finally:
        range_pop()
