"""Deferred BatchNorm: running statistics per *mini-batch*, not per micro-batch.

Parity: ``torchgpipe/batchnorm.py:17-155``.  With ``chunks`` micro-batches a
plain BatchNorm would update its running statistics ``chunks`` times per
step with small-batch estimates.  ``DeferredBatchNorm`` normalises each
micro-batch with its own statistics (like BatchNorm in training) but only
*accumulates* per-channel ``Σx`` and ``Σx²`` (buffers ``sum`` /
``sum_squares``, kept for state-dict compatibility) and commits one
running-statistics update when the last micro-batch of the mini-batch has
been tracked.  Tracking is skipped during checkpoint recomputation.

MI355X implementation:

* K1 ``dbn_track``: one HIP kernel reads the micro-batch once (16-byte
  vector loads, wave64 shuffle + LDS reduction per block, one fp32 atomic
  per block and channel) instead of PyTorch's ``sum`` / ``pow`` / ``sum`` /
  ``add_`` ×2 sequence.
* K2 ``dbn_commit``: one HIP kernel turns the sums into mean / variance,
  applies the EMA and zeroes the accumulators.

Deliberate fixes over the reference:

* the committed variance is **unbiased** (Bessel-corrected), matching
  ``nn.BatchNorm``'s running_var, instead of the biased ``E[x²]−E[x]²``;
* the commit fires after the number of micro-batches *actually* produced by
  ``scatter`` (``Tensor.chunk`` can yield fewer than ``chunks``), so the
  commit window never drifts: ``GPipe`` sets ``expected_chunks`` per forward
  via :func:`set_micro_batches`.
"""
from typing import Optional, TypeVar, cast

import torch
from torch import Tensor, nn
import torch.nn.functional as F
from torch.nn.modules.batchnorm import _BatchNorm

from torchgpipe_amd.checkpoint import is_recomputing
from torchgpipe_amd.ops import dbn as dbn_ops

__all__ = ['DeferredBatchNorm']

TModule = TypeVar('TModule', bound=nn.Module)


class DeferredBatchNorm(_BatchNorm):
    sum: Tensor
    sum_squares: Tensor

    def __init__(self, num_features: int, eps: float = 1e-5,
                 momentum: Optional[float] = 0.1, affine: bool = True,
                 chunks: int = 1) -> None:
        super().__init__(num_features, eps, momentum, affine, track_running_stats=True)
        self.register_buffer('sum', torch.zeros_like(self.running_mean))
        self.register_buffer('sum_squares', torch.zeros_like(self.running_var))
        self.counter = 0
        self.tracked = 0
        self.chunks = chunks
        self.expected_chunks: Optional[int] = None

    def reset_running_stats(self) -> None:
        """Reset running statistics *and* the deferred accumulators.

        ``_BatchNorm.reset_running_stats`` does not know ``sum`` / ``sum_squares``;
        without this, a DeferredBatchNorm materialised from the meta device
        (``utils.meta.materialize``) would commit allocator garbage.
        """
        super().reset_running_stats()
        if hasattr(self, 'sum'):
            self.sum.zero_()
            self.sum_squares.zero_()
        self.counter = 0
        self.tracked = 0

    def _check_input_dim(self, input: Tensor) -> None:
        if input.dim() <= 2:
            raise ValueError('expected at least 3D input (got %dD input)' % input.dim())

    def _track(self, input: Tensor) -> bool:
        dbn_ops.track(input, self.sum, self.sum_squares)
        self.counter += input.numel() // input.size(1)
        self.tracked += 1
        target = self.expected_chunks if self.expected_chunks is not None else self.chunks
        return self.tracked >= target

    def _commit(self) -> None:
        self.num_batches_tracked += 1
        if self.momentum is None:
            factor = 1.0 / float(self.num_batches_tracked)
        else:
            factor = float(self.momentum)
        dbn_ops.commit(self.sum, self.sum_squares, self.running_mean, self.running_var,
                       self.counter, factor)
        self.counter = 0
        self.tracked = 0

    def forward(self, input: Tensor) -> Tensor:  # type: ignore[override]
        self._check_input_dim(input)
        if not self.training:
            return F.batch_norm(input, self.running_mean, self.running_var,
                                self.weight, self.bias, False, 0.0, self.eps)
        if not is_recomputing():
            if self._track(input):
                self._commit()
        return F.batch_norm(input, None, None, self.weight, self.bias, True, 0.0, self.eps)

    @classmethod
    def convert_deferred_batch_norm(cls, module: TModule, chunks: int = 1) -> TModule:
        """Recursively replace ``nn.BatchNorm*`` (with running stats) by DeferredBatchNorm.

        Parameters and running buffers are shared, not copied.
        """
        if isinstance(module, DeferredBatchNorm) and module.chunks is chunks:
            return module
        out: nn.Module = module
        if isinstance(module, _BatchNorm) and module.track_running_stats:
            out = DeferredBatchNorm(module.num_features, module.eps, module.momentum,
                                    module.affine, chunks)
            if module.affine:
                out.register_parameter('weight', module.weight)
                out.register_parameter('bias', module.bias)
            out.register_buffer('running_mean', module.running_mean)
            out.register_buffer('running_var', module.running_var)
            out.register_buffer('num_batches_tracked', module.num_batches_tracked)
        for name, child in module.named_children():
            out.add_module(name, cls.convert_deferred_batch_norm(child, chunks))
        return cast(TModule, out)


def set_micro_batches(module: nn.Module, count: Optional[int]) -> None:
    """Tell every DeferredBatchNorm in ``module`` how many micro-batches this step has."""
    for m in module.modules():
        if isinstance(m, DeferredBatchNorm):
            m.expected_chunks = count
