"""Utilities: GPU timing, profiler ranges, runtime configuration."""
from .config import BY_NAME, KNOBS, describe  # noqa: F401
from .profiling import range_pop, range_push, trace_range  # noqa: F401
from .timing import GpuTimer, benchmark  # noqa: F401
from .graphs import CapturedCall  # noqa: F401
