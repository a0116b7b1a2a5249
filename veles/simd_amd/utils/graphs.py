"""HIP-graph capture of launch-bound sequences of veles ops.

The library's kernels launch on the caller's stream and take their scratch
from a caching pool, so after one warm-up run (which fills the pool and the
FFT twiddle / wavelet caches) a sequence of ops contains no allocation, no
synchronous copy and no host decision that depends on data -- it can be
captured once into a HIP graph (torch.cuda.CUDAGraph) and replayed with one
launch.  This replaces a tracing compiler for the short, launch-bound
pipelines the reference runs as loops of tiny calls (e.g. a filter bank over
many small signals).

Calls that need more than 1 MiB of scratch in one allocation (partitioned
overlap-save for filters past one block, tiled pyramids of long rows, the
four-step FFT) raise an error when captured: keep them outside the graph.

    g = CapturedCall(lambda x: ops.conv1d(ops.swt(x, "daubechies", 8, 3)[1], h), x0)
    y = g(x1)    # copies x1 into the static input, replays, returns the output
"""
from __future__ import annotations

from typing import Callable, Sequence

import torch


class CapturedCall:
    """Capture `fn(*static_inputs)` into a HIP graph after `warmup` eager runs.

    Calling the object copies new inputs (same shapes / dtypes) into the
    static input tensors, replays the graph, and returns the static outputs
    (which are overwritten by the next call: clone them to keep them).
    """

    def __init__(self, fn: Callable, *static_inputs: torch.Tensor, warmup: int = 2):
        if not torch.cuda.is_available():
            raise RuntimeError("CapturedCall needs a GPU")
        self.fn = fn
        self.inputs: Sequence[torch.Tensor] = [t.clone() for t in static_inputs]
        # Warm up on the stream that will be captured (fills the twiddle /
        # filter caches); inside the capture the library's scratch comes
        # from stream-ordered graph allocations (csrc/runtime ScratchPool).
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                fn(*self.inputs)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=side):
            self.outputs = fn(*self.inputs)

    def __call__(self, *inputs: torch.Tensor):
        for dst, src in zip(self.inputs, inputs):
            dst.copy_(src, non_blocking=True)
        self.graph.replay()
        return self.outputs
