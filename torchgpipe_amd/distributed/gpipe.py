"""``DistributedGPipe``: the reference's multi-process API on the RCCL engine.

API parity with ``torchgpipe/distributed/gpipe.py:26-275``:

* ``get_module_partition(module, rank, balance, device)``
* ``DistributedGPipe(module, rank, workers, balance, microbatch_chunks, *,
  device=None, deferred_batch_norm=False)`` with ``forward(batch)`` (rank 0
  passes the mini-batch, the others ``None``; returns the list of
  per-micro-batch outputs) and ``backward(losses)`` (the last rank passes one
  loss per micro-batch, the others ``None``);
* ``DistributedGPipeDataLoader`` that hands the data to rank 0 and ships the
  target to the last rank.

Differences (all improvements): tensors go GPU→GPU over RCCL instead of
CPU-staged RPC; activation checkpointing (``checkpoint=``), skip connections
and deferred BatchNorm work; ``workers`` (rank → name) is only used for
naming since ranks address each other through ``torch.distributed``.
"""
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor, nn
import torch.distributed as dist

from torchgpipe_amd.gpipe import BalanceError, check_balance, partition_layers, \
    recommend_auto_balance, verify_module
from torchgpipe_amd.parallel.p2p import P2P
from torchgpipe_amd.parallel.stage import PipelineStage

__all__ = ['DistributedGPipe', 'DistributedGPipeDataLoader', 'get_module_partition']

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]


def get_module_partition(module: nn.Sequential, rank: int, balance: Iterable[int],
                         device: Optional[torch.device]) -> nn.Sequential:
    """The ``rank``-th partition of ``module`` under ``balance`` (moved to ``device``)."""
    balance = list(balance)
    check_balance(module, balance)
    if not 0 <= rank < len(balance):
        raise RuntimeError('module and balance mismatch')
    partition = nn.Sequential(partition_layers(module, balance)[rank])
    if device is not None:
        partition.to(device)
    return partition


class DistributedGPipe:
    """One pipeline stage per process; see module docstring."""

    chunks: int = 1

    def __init__(self, module: nn.Sequential, rank: int, workers: Optional[Dict[int, str]] = None,
                 balance: Optional[Iterable[int]] = None, microbatch_chunks: int = chunks, *,
                 device: Optional[torch.device] = None, deferred_batch_norm: bool = False,
                 checkpoint: str = 'never', group: Optional[dist.ProcessGroup] = None,
                 timeout: Optional[float] = None) -> None:
        microbatch_chunks = int(microbatch_chunks)
        if balance is None:
            raise ValueError(recommend_auto_balance('balance is required'))
        if microbatch_chunks <= 0:
            raise ValueError('number of chunks must be positive integer')
        verify_module(module)
        balance = list(balance)
        try:
            check_balance(module, balance)
        except BalanceError as exc:
            raise ValueError(recommend_auto_balance(str(exc)))

        self.rank = rank
        self.workers = workers or {r: f'worker{r}' for r in range(len(balance))}
        self.world_size = len(self.workers)
        self.name = self.workers[rank]
        self.chunks = microbatch_chunks
        self.device = device if device is not None else torch.device('cpu')
        self.stage = PipelineStage(module, balance, rank=rank, device=self.device,
                                   chunks=microbatch_chunks, checkpoint=checkpoint, group=group,
                                   deferred_batch_norm=deferred_batch_norm, timeout=timeout)
        self.module = self.stage.partition
        self._outputs: List[TensorOrTensors] = []

    def model(self) -> nn.Sequential:
        return self.module

    def parameters(self) -> Iterator[nn.Parameter]:
        return self.module.parameters()

    def train(self, mode: bool = True) -> 'DistributedGPipe':
        self.stage.train(mode)
        return self

    def eval(self) -> 'DistributedGPipe':
        return self.train(False)

    def forward(self, batch: Optional[TensorOrTensors]) -> List[TensorOrTensors]:
        if batch is not None and self.rank != 0:
            raise AssertionError('only the first stage receives the mini-batch')
        self._outputs = self.stage.forward(batch)
        return self._outputs

    __call__ = forward

    def backward(self, losses: Optional[Sequence[Tensor]]) -> None:
        if losses is not None and self.rank != self.world_size - 1:
            raise AssertionError('only the last stage computes losses')
        self.stage.backward(losses)
        self._outputs = []


class DistributedGPipeDataLoader:
    """Stage-aware loader: rank 0 yields ``(data, None)`` and ships the target to the
    last stage, which yields ``(None, target)``; middle stages yield ``(None, None)``.

    The target crosses over RCCL (GPU-direct) instead of CPU-staged RPC.  Pass
    ``pipeline`` to reuse its transport (and its per-link communicators).
    """

    def __init__(self, data_loader: Optional[Iterable], rank: int, chunks: int,
                 num_iterations: int, last_stage: bool, last_stage_name: str = '', *,
                 last_rank: Optional[int] = None, device: Optional[torch.device] = None,
                 pipeline: Optional[DistributedGPipe] = None) -> None:
        self._data_loader = data_loader
        self._rank = rank
        self._chunks = chunks
        self._num_iterations = num_iterations
        self._last_stage = last_stage
        self._last_stage_name = last_stage_name
        world = dist.get_world_size() if dist.is_initialized() else 1
        self._last_rank = world - 1 if last_rank is None else last_rank
        self._device = device or (pipeline.device if pipeline is not None else torch.device('cpu'))
        self._p2p: Optional[P2P] = pipeline.stage.p2p if pipeline is not None else None
        if self._p2p is None and dist.is_initialized():
            # new_group is collective: every rank builds the control group here.
            ctrl = (dist.group.WORLD if dist.get_backend() == 'gloo'
                    else dist.new_group(backend='gloo'))
            self._p2p = P2P(self._device, ctrl_group=ctrl)

    def _transport(self) -> P2P:
        if self._p2p is None:
            raise RuntimeError('torch.distributed must be initialized to ship targets')
        return self._p2p

    def _first_stage_iter(self) -> Iterator[Tuple[Optional[Tensor], Optional[Tensor]]]:
        assert self._data_loader is not None
        for it, (data, target) in zip(range(self._num_iterations), self._data_loader):
            if self._last_rank != self._rank:
                p2p = self._transport()
                p2p.send([target.to(self._device)], self._last_rank, ('target', it), cache=False)
                # Complete the hand-off before handing control back: a send still
                # pending when its transport is released would be dropped.
                p2p.flush()
                yield data, None
            else:
                yield data, target

    def _last_stage_iter(self) -> Iterator[Tuple[Optional[Tensor], Optional[Tensor]]]:
        for it in range(self._num_iterations):
            # One-shot key: every target carries its own metadata (shapes may
            # vary per iteration) and nothing accumulates in the metadata cache.
            msg = self._transport().recv(0, ('target', it), cache=False)
            (target,) = msg.wait()
            yield None, target.detach()

    def _middle_stage_iter(self) -> Iterator[Tuple[Optional[Tensor], Optional[Tensor]]]:
        for _ in range(self._num_iterations):
            yield None, None

    def __iter__(self) -> Iterator[Tuple[Optional[Tensor], Optional[Tensor]]]:
        if self._rank == 0:
            return self._first_stage_iter()
        if self._last_stage:
            return self._last_stage_iter()
        return self._middle_stage_iter()

    def __len__(self) -> int:
        return self._num_iterations
