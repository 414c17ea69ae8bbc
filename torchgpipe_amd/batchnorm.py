"""Deferred BatchNorm: running statistics per *mini-batch*, not per micro-batch.

Parity: ``torchgpipe/batchnorm.py:17-155``.  With ``chunks`` micro-batches a
plain BatchNorm would update its running statistics ``chunks`` times per
step with small-batch estimates.  ``DeferredBatchNorm`` normalises each
micro-batch with its own statistics (like BatchNorm in training) but only
*accumulates* per-channel ``Σx`` and ``Σx²`` (buffers ``sum`` /
``sum_squares``, kept for state-dict compatibility) and commits one
running-statistics update when the last micro-batch of the mini-batch has
been tracked.  Tracking is skipped during checkpoint recomputation.

MI355X implementation (fp32 GPU tensors):

* Forward = one native BatchNorm-train op (``tgpipe::bn_train_forward``,
  ``csrc/batchnorm.hip``): per-(image, channel) (mean, M2) partials, a finalize
  that merges them with Chan's formula in fp64 into the micro-batch statistics
  used for normalisation *and* folds them into the mini-batch accumulators, and
  one normalising pass -- the input is read twice (statistics, normalisation)
  instead of three times (tracking kernel + MIOpen BatchNorm), and no
  E[x²]−E[x]² cancellation exists anywhere (means of 1e3 with std 1e-1 keep
  ``running_var`` to 1e-4 relative).  The backward is native too
  (``bn_train_backward``).
* The accumulators are an fp64 ``[3][C]`` (count, mean, M2) buffer, not part of
  the state dict; ``dbn_commit64`` turns them into the running-statistics EMA
  and zeroes them.  ``sum`` / ``sum_squares`` stay registered (and zero) so the
  reference's state-dict keys are unchanged.
* CPU tensors: the same Chan accumulation in fp64 PyTorch ops (the oracle).

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
from torchgpipe_amd.ops import _ext

__all__ = ['DeferredBatchNorm']

TModule = TypeVar('TModule', bound=nn.Module)


class _BNTrain(torch.autograd.Function):
    """Native BatchNorm-train forward/backward; folds statistics into ``acc`` if given."""

    @staticmethod
    def forward(ctx, x: Tensor, weight: Optional[Tensor], bias: Optional[Tensor],  # type: ignore[override]
                acc: Optional[Tensor], eps: float) -> Tensor:
        y, mean, invstd, sums = _ext.require(x).bn_train_forward(x, weight, bias, acc, eps)
        ctx.save_for_backward(x, mean, invstd, sums, weight)
        return y

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        x, mean, invstd, sums, weight = ctx.saved_tensors
        dx, dgamma, dbeta = _ext.require(dy).bn_train_backward(dy, x, mean, invstd, sums,
                                                                weight)
        return (dx, dgamma if ctx.needs_input_grad[1] else None,
                dbeta if ctx.needs_input_grad[2] else None, None, None)


def _chan_merge_(acc: Tensor, x: Tensor) -> None:
    """Fold x's per-channel (count, mean, M2) into acc [3][C] (fp64 PyTorch ops)."""
    dims = [0] + list(range(2, x.dim()))
    xd = x.detach().double()
    nb = float(xd.numel() // xd.size(1))
    mb = xd.mean(dims)
    m2b = ((xd - mb.view(1, -1, *([1] * (x.dim() - 2)))) ** 2).sum(dims)
    na = acc[0]
    n = na + nb
    delta = mb - acc[1]
    acc[1] += delta * nb / n
    acc[2] += m2b + delta * delta * na * nb / n
    acc[0] = n


class DeferredBatchNorm(_BatchNorm):
    sum: Tensor
    sum_squares: Tensor
    acc: Tensor

    def __init__(self, num_features: int, eps: float = 1e-5,
                 momentum: Optional[float] = 0.1, affine: bool = True,
                 chunks: int = 1) -> None:
        super().__init__(num_features, eps, momentum, affine, track_running_stats=True)
        self.register_buffer('sum', torch.zeros_like(self.running_mean))
        self.register_buffer('sum_squares', torch.zeros_like(self.running_var))
        # (count, mean, M2) of the mini-batch so far; fp64, outside the state dict
        self.register_buffer('acc', torch.zeros(3, num_features, dtype=torch.float64),
                             persistent=False)
        self.counter = 0
        self.tracked = 0
        self.chunks = chunks
        self.expected_chunks: Optional[int] = None

    def reset_running_stats(self) -> None:
        """Reset running statistics *and* the deferred accumulators.

        ``_BatchNorm.reset_running_stats`` does not know ``sum`` / ``sum_squares`` /
        ``acc``; without this, a DeferredBatchNorm materialised from the meta device
        (``utils.meta.materialize``) would commit allocator garbage.
        """
        super().reset_running_stats()
        for name in ('sum', 'sum_squares', 'acc'):
            if hasattr(self, name):
                getattr(self, name).zero_()
        self.counter = 0
        self.tracked = 0

    def _check_input_dim(self, input: Tensor) -> None:
        if input.dim() <= 2:
            raise ValueError('expected at least 3D input (got %dD input)' % input.dim())

    def _native(self, input: Tensor) -> bool:
        return (input.is_cuda and input.dtype == torch.float32
                and self.running_mean.dtype == torch.float32 and _ext.available())

    def _tracked_one(self, input: Tensor) -> bool:
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
        if self.acc.is_cuda and self.running_mean.dtype == torch.float32:
            _ext.require(self.acc).dbn_commit64(self.acc, self.running_mean, self.running_var,
                                                factor)
        else:
            with torch.no_grad():
                n, mean, m2 = self.acc[0], self.acc[1], self.acc[2]
                var = torch.where(n > 1, m2 / (n - 1).clamp(min=1), torch.zeros_like(m2))
                self.running_mean.mul_(1 - factor).add_(mean.to(self.running_mean.dtype),
                                                        alpha=factor)
                self.running_var.mul_(1 - factor).add_(var.to(self.running_var.dtype),
                                                       alpha=factor)
                self.acc.zero_()
        self.counter = 0
        self.tracked = 0

    def forward(self, input: Tensor) -> Tensor:  # type: ignore[override]
        self._check_input_dim(input)
        if not self.training:
            return F.batch_norm(input, self.running_mean, self.running_var,
                                self.weight, self.bias, False, 0.0, self.eps)
        track = not is_recomputing()
        if self._native(input):
            out = _BNTrain.apply(input.contiguous(), self.weight, self.bias,
                                 self.acc if track else None, float(self.eps))
        else:
            if track:
                _chan_merge_(self.acc, input)
            out = F.batch_norm(input, None, None, self.weight, self.bias, True, 0.0, self.eps)
        if track and self._tracked_one(input):
            self._commit()
        return out

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
