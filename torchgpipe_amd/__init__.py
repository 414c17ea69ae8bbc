"""torchgpipe_amd — an MI355X-native GPipe pipeline-parallel training engine.

Public API (compatible with ``torchgpipe``):

* :class:`GPipe` — single-process pipeline over several devices
* :func:`is_checkpointing`, :func:`is_recomputing`
* :mod:`torchgpipe_amd.skip` — ``@skippable`` long skip connections
* :mod:`torchgpipe_amd.balance` — ``balance_by_time`` / ``balance_by_size``
* :mod:`torchgpipe_amd.batchnorm` — ``DeferredBatchNorm``
* :mod:`torchgpipe_amd.distributed` — multi-process pipeline (one rank per GPU,
  RCCL point-to-point over xGMI): ``DistributedGPipe``,
  ``DistributedGPipeDataLoader``
"""
from torchgpipe_amd.__version__ import __version__
from torchgpipe_amd.checkpoint import is_checkpointing, is_recomputing
from torchgpipe_amd.gpipe import GPipe

__all__ = ['GPipe', 'is_checkpointing', 'is_recomputing', '__version__']
