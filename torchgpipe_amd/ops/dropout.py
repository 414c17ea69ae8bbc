"""Inverted dropout with explicit Philox ``(seed, offset)`` (K4).

:class:`Dropout` (elementwise) and :class:`Dropout2d` (whole channels) are
drop-in replacements for ``nn.Dropout`` / ``nn.Dropout2d`` used by the model
zoo.  Their randomness comes from :func:`~torchgpipe_amd.utils.rng.philox_pair`,
so checkpoint recomputation replays the cell's recorded ``(seed, offset)``
pairs from its RNG tape instead of restoring global generator state from an
autograd thread (the reference's ``fork_rng``, ``torchgpipe/checkpoint.py:191-231``).
The elementwise kernel stores no mask: backward regenerates it from the pair.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor, nn

from torchgpipe_amd.ops import _ext
from torchgpipe_amd.ops.fused import _signed64
from torchgpipe_amd.ops.philox import uniform
from torchgpipe_amd.utils.rng import philox_draw

__all__ = ['dropout', 'Dropout', 'dropout2d', 'Dropout2d', 'convert_dropout']


def _reference(x: Tensor, p: float, seed: int, offset: int) -> Tensor:
    keep = uniform(x.numel(), seed, offset).to(x.device).view_as(x) >= p
    return x * keep.to(x.dtype) / (1.0 - p)


class _Dropout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, p: float, seed: int, offset: int,  # type: ignore[override]
                rng: Optional[Tensor] = None) -> Tensor:
        ctx.p, ctx.seed, ctx.offset, ctx.rng = p, seed, offset, rng
        return _ext.require(x).dropout(x, p, seed, offset, rng)

    @staticmethod
    def backward(ctx, dy: Tensor) -> Tuple:  # type: ignore[override]
        # The same mask and scale apply to the gradient.
        return _ext.require(dy).dropout(dy.contiguous(), ctx.p, ctx.seed, ctx.offset,
                                        ctx.rng), None, None, None, None


def dropout(x: Tensor, p: float = 0.5, training: bool = True) -> Tensor:
    if not training or p == 0.0:
        return x
    if p >= 1.0:
        return x * 0.0
    seed, offset, rng = philox_draw(x.device, x.numel())
    if x.is_cuda and x.dtype == torch.float32:
        return _Dropout.apply(x.contiguous(), float(p), _signed64(seed), _signed64(offset), rng)
    if rng is not None:
        raise RuntimeError('dropout: a device Philox slot needs the fp32 GPU kernel')
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


class _Dropout2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, scale: Tensor) -> Tensor:  # type: ignore[override]
        ctx.save_for_backward(scale)
        return x * scale

    @staticmethod
    def backward(ctx, dy: Tensor) -> Tuple:  # type: ignore[override]
        (scale,) = ctx.saved_tensors
        return dy * scale, None


def dropout2d(x: Tensor, p: float = 0.5, training: bool = True) -> Tensor:
    """Channel dropout: each (image, channel) plane is kept with probability ``1 - p``."""
    if not training or p == 0.0:
        return x
    if p >= 1.0:
        return x * 0.0
    planes = x.shape[0] * x.shape[1]
    seed, offset, rng = philox_draw(x.device, planes)
    if x.is_cuda:
        u = _ext.require(x).philox_uniform(planes, _signed64(seed), _signed64(offset), x.device,
                                           rng)
    else:
        u = uniform(planes, seed, offset)
    keep = (u >= p).to(x.dtype).view(x.shape[0], x.shape[1], *([1] * (x.dim() - 2)))
    return _Dropout2d.apply(x, keep.to(x.device) / (1.0 - p))


class Dropout2d(nn.Module):
    """``nn.Dropout2d`` on tape-replayable Philox draws."""

    def __init__(self, p: float = 0.5) -> None:
        super().__init__()
        if not 0.0 <= p <= 1.0:
            raise ValueError(f'dropout probability has to be between 0 and 1, but got {p}')
        self.p = p

    def extra_repr(self) -> str:
        return f'p={self.p}'

    def forward(self, x: Tensor) -> Tensor:  # type: ignore[override]
        return dropout2d(x, self.p, self.training)


def convert_dropout(module: nn.Module) -> nn.Module:
    """Replace every ``nn.Dropout`` / ``nn.Dropout2d`` in ``module`` (exact types, in place;
    ``module`` itself too) by :class:`Dropout` / :class:`Dropout2d` with the same ``p`` and
    training mode, and return the module.

    ``GPipe(..., philox_dropout=True)`` / ``PipelineStage(..., philox_dropout=True)`` call
    it: the user's dropout layers then draw explicit Philox pairs that a checkpointed
    cell's RNG tape replays during recomputation, instead of the global-generator fork /
    restore of the reference's checkpointing (``torchgpipe/checkpoint.py:191-231``), which
    mutates process-global state from autograd threads.  The masks come from another
    random stream than ``torch.nn.functional.dropout``'s, so the result is not bitwise the
    plain model's under the same ``torch.manual_seed`` (the reason it is opt-in).
    """
    def swap(m: nn.Module) -> nn.Module:
        if type(m) is nn.Dropout:
            new: nn.Module = Dropout(m.p)
        elif type(m) is nn.Dropout2d:
            new = Dropout2d(m.p)
        else:
            return m
        new.train(m.training)
        return new

    for name, child in list(module.named_children()):
        swapped = swap(child)
        if swapped is not child:
            setattr(module, name, swapped)
        else:
            convert_dropout(child)
    return swap(module)
