"""Multi-process pipeline parallelism (one process per GPU, RCCL over xGMI).

Parity with ``torchgpipe.distributed`` (the reference's RPC-based fork
addition): :class:`DistributedGPipe`, :class:`DistributedGPipeDataLoader`,
:func:`get_module_partition` and the :mod:`.context` mailboxes.
"""
from torchgpipe_amd.distributed import context
from torchgpipe_amd.distributed.gpipe import (DistributedGPipe, DistributedGPipeDataLoader,
                                              get_module_partition)

__all__ = ['DistributedGPipe', 'DistributedGPipeDataLoader', 'get_module_partition', 'context']
