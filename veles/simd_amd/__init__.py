"""veles.simd_amd -- MI355X-native rebuild of veles.simd.

Layers (bottom -> top):
  * ``_native/libvelessimd.so``: HIP/CDNA4 kernels for gfx950, the C++ runtime
    and the source-compatible C API (``include/simd/*.h``);
  * :mod:`veles.simd_amd.capi`: numpy access to that C API (host pointers);
  * :mod:`veles.simd_amd.ops`: PyTorch custom ops (``torch.ops.veles.*``);
  * :mod:`veles.simd_amd.parallel`: one-process-per-GPU data / row / sequence
    parallelism over RCCL (``torch.distributed`` backend "nccl");
  * :mod:`veles.simd_amd.models`: composed DSP pipelines as ``nn.Module``;
  * :mod:`veles.simd_amd.utils`: timing, profiling ranges, env config.
"""
from . import _lib
from ._lib import NativeLibraryMissing, VelesError, available, gpu_available

__version__ = "0.1.0"

__all__ = ["NativeLibraryMissing", "VelesError", "available", "gpu_available",
           "__version__"]
