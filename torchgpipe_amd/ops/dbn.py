"""DeferredBatchNorm statistics ops (K1 ``dbn_track`` / K2 ``dbn_commit``).

GPU: HIP kernels from ``csrc/kernels.hip``.  CPU: the reference math
(``torchgpipe/batchnorm.py:45-85``) with the unbiased-variance fix.
"""
import torch
from torch import Tensor

from torchgpipe_amd.ops import _ext

__all__ = ['track', 'commit']


def track(input: Tensor, sum: Tensor, sum_squares: Tensor) -> None:
    """``sum += Σ_{n,spatial} x``, ``sum_squares += Σ x²`` per channel (no autograd)."""
    x = input.detach()
    if x.is_cuda and x.dtype == torch.float32 and sum.dtype == torch.float32:
        _ext.require(x).dbn_track(x.contiguous(), sum, sum_squares)
        return
    dims = [0] + list(range(2, x.dim()))
    with torch.no_grad():
        xf = x.to(sum.dtype)
        sum += xf.sum(dims)
        sum_squares += (xf * xf).sum(dims)


def commit(sum: Tensor, sum_squares: Tensor, running_mean: Tensor, running_var: Tensor,
           count: int, momentum: float) -> None:
    """EMA update of the running statistics from the accumulated sums; zero the sums."""
    if sum.is_cuda and sum.dtype == torch.float32 and running_mean.dtype == torch.float32:
        _ext.require(sum).dbn_commit(sum, sum_squares, running_mean, running_var,
                                     float(count), float(momentum))
        return
    with torch.no_grad():
        mean = sum.double() / count
        var = (sum_squares.double() / count - mean * mean).clamp_(min=0)
        if count > 1:
            var = var * (count / (count - 1))
        running_mean.mul_(1 - momentum).add_(mean.to(running_mean.dtype), alpha=momentum)
        running_var.mul_(1 - momentum).add_(var.to(running_var.dtype), alpha=momentum)
        sum.zero_()
        sum_squares.zero_()
