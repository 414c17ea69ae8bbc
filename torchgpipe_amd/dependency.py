"""Arbitrary ordering edges between two autograd lanes (Fork / Join).

Parity: ``torchgpipe/dependency.py:12-48``.  ``fork(x)`` returns ``(x', p)``
where ``p`` is a phony that depends on ``x``; ``join(y, p)`` returns ``y'``
that depends on ``p``.  In the backward pass this forces ``y``'s gradient
path to be processed before ``x``'s — the pipeline uses it to make micro-batch
``i-1`` back-propagate after micro-batch ``i`` on every partition, and the
skip subsystem uses it to tie hidden portal tensors to a micro-batch lane.

Both are value-identities and no-ops when grad is disabled.
"""
from typing import List, Tuple

import torch
from torch import Tensor

from torchgpipe_amd.phony import get_phony

__all__: List[str] = []


class Fork(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input: Tensor) -> Tuple[Tensor, Tensor]:  # type: ignore[override]
        return input.detach(), get_phony(input.device, requires_grad=False).detach()

    @staticmethod
    def backward(ctx, grad: Tensor, _grad_phony: Tensor) -> Tensor:  # type: ignore[override]
        return grad


class Join(torch.autograd.Function):
    @staticmethod
    def forward(ctx, input: Tensor, phony: Tensor) -> Tensor:  # type: ignore[override]
        return input.detach()

    @staticmethod
    def backward(ctx, grad: Tensor) -> Tuple[Tensor, None]:  # type: ignore[override]
        return grad, None


def fork(input: Tensor) -> Tuple[Tensor, Tensor]:
    """Branch a phony lane out of ``input``'s autograd lane."""
    if torch.is_grad_enabled() and input.requires_grad:
        return Fork.apply(input)
    return input, get_phony(input.device, requires_grad=False)


def join(input: Tensor, phony: Tensor) -> Tensor:
    """Merge ``phony``'s lane into ``input``'s autograd lane."""
    if torch.is_grad_enabled() and (input.requires_grad or phony.requires_grad):
        return Join.apply(input, phony)
    return input
