"""GPU-event timing helpers (the reference times with std::chrono around a
host loop, tests/benchmark.inc:74-107; on the GPU we time with HIP events on
the stream that runs the kernels)."""
from __future__ import annotations

import statistics
import time
from typing import Callable

import torch


class GpuTimer:
    """Context manager measuring elapsed GPU time on the current stream."""

    def __init__(self):
        self.ms = float("nan")
        self._cuda = torch.cuda.is_available()

    def __enter__(self):
        if self._cuda:
            self._e0 = torch.cuda.Event(enable_timing=True)
            self._e1 = torch.cuda.Event(enable_timing=True)
            self._e0.record()
        else:
            self._t0 = time.perf_counter()
        return self

    def __exit__(self, *exc):
        if self._cuda:
            self._e1.record()
            self._e1.synchronize()
            self.ms = self._e0.elapsed_time(self._e1)
        else:
            self.ms = (time.perf_counter() - self._t0) * 1e3
        return False


def benchmark(fn: Callable[[], object], reps: int = 10, warmup: int = 2,
              rounds: int = 5) -> dict:
    """Median / min per-call milliseconds of fn over `rounds` timed batches."""
    for _ in range(warmup):
        fn()
    per = []
    for _ in range(rounds):
        with GpuTimer() as t:
            for _ in range(reps):
                fn()
        per.append(t.ms / reps)
    return {"median_ms": statistics.median(per), "min_ms": min(per), "rounds": per}
