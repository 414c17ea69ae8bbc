"""Elementwise inverted dropout with explicit Philox ``(seed, offset)`` (K4).

Unlike ``nn.Dropout`` it stores no mask: backward regenerates it from the
saved ``(seed, offset)``, and checkpoint recomputation replays the same pair
from the cell's RNG tape instead of restoring global generator state.
"""
from typing import Tuple

import torch
from torch import Tensor, nn

from torchgpipe_amd.ops import _ext
from torchgpipe_amd.ops.fused import _signed64
from torchgpipe_amd.ops.philox import uniform
from torchgpipe_amd.utils.rng import philox_pair

__all__ = ['dropout', 'Dropout']


def _reference(x: Tensor, p: float, seed: int, offset: int) -> Tensor:
    keep = uniform(x.numel(), seed, offset).to(x.device).view_as(x) >= p
    return x * keep.to(x.dtype) / (1.0 - p)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, p: float, seed: int, offset: int) -> Tensor:  # type: ignore[override]
        ctx.p, ctx.seed, ctx.offset = p, seed, offset
        return _ext.require(x).dropout(x, p, seed, offset)

    @staticmethod
    def backward(ctx, dy: Tensor) -> Tuple:  # type: ignore[override]
        # The same mask and scale apply to the gradient.
        return _ext.require(dy).dropout(dy.contiguous(), ctx.p, ctx.seed, ctx.offset), \
            None, None, None


def dropout(x: Tensor, p: float = 0.5, training: bool = True) -> Tensor:
    if not training or p == 0.0:
        return x
    if p >= 1.0:
        return x * 0.0
    seed, offset = philox_pair(x.device, x.numel())
    if x.is_cuda and x.dtype == torch.float32:
        return _Dropout.apply(x.contiguous(), float(p), _signed64(seed), _signed64(offset))
    return _reference(x, p, seed, offset)


class Dropout(nn.Module):
    def __init__(self, p: float = 0.5) -> None:
        super().__init__()
        if not 0.0 <= p <= 1.0:
            raise ValueError(f'dropout probability has to be between 0 and 1, but got {p}')
        self.p = p

    def extra_repr(self) -> str:
        return f'p={self.p}'

    def forward(self, x: Tensor) -> Tensor:  # type: ignore[override]
        return dropout(x, self.p, self.training)
