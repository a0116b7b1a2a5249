"""Multi-GPU execution: one process per GPU, RCCL over xGMI.

* :mod:`comm` -- process-group setup (``torch.distributed``, backend "nccl"
  = RCCL on ROCm, "gloo" on CPU), shard arithmetic, padded all-gather.
* :mod:`data_parallel` -- batch sharding of any op (D2).
* :mod:`tensor_parallel` -- row-split batched SGEMM with overlapped
  broadcast / all-gather (D3).
* :mod:`context_parallel` -- long-signal convolution / SWT with halo exchange
  (D4).
"""
from . import comm, context_parallel, data_parallel, tensor_parallel  # noqa: F401
from .comm import DistContext, all_gather_rows, init, shard_range  # noqa: F401
from .context_parallel import cp_conv1d, cp_swt  # noqa: F401
from .data_parallel import dp_apply, local_shard  # noqa: F401
from .tensor_parallel import rowsplit_bmm  # noqa: F401
