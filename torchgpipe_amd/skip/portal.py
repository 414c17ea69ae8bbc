"""Portals: carry a skip tensor outside the autograd graph.

Parity: ``torchgpipe/skip/portal.py:22-227``.  A skip tensor stashed in
partition ``j`` and popped in ``k`` would, if passed through the pipeline as a
regular tensor, be copied through every intermediate partition and kept
alive there.  A portal instead *hides* it:

* ``PortalBlue`` (stash side) consumes the tensor and returns a phony that is
  joined into the micro-batch lane; its backward emits the gradient that the
  pop side deposited.
* ``PortalCopy`` moves the hidden tensor directly from ``j``'s device to
  ``k``'s device (one xGMI hop, on the copy streams) and the gradient back.
* ``PortalOrange`` (pop side) returns the hidden tensor; its backward stores
  the incoming gradient into the portal.

A reference count ("tensor life") frees the hidden tensor as soon as its
last user — which depends on whether the cell is checkpointed — has run::

    1 [x] blue()                 7 [ ] orange() (recomputed)
    2 [ ]   PortalBlue.forward    8 [x]   PortalOrange.forward (recomputed)
    3 [ ] copy()                  9 [ ]   PortalOrange.backward
    4 [ ]   PortalCopy.forward   10 [ ] PortalCopy.backward
    5 [ ] orange()               11 [x] blue() (recomputed)
    6 [x]   PortalOrange.forward 12 [ ]   PortalBlue.forward (recomputed)
                                 13 [ ]   PortalBlue.backward

([x] = consumes one life.)  Checkpointed cells need life 3 (freed at 8),
others life 2 (freed at 6); the recomputed stash resets life to 1.
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from torchgpipe_amd.copy import Copy
from torchgpipe_amd.phony import get_phony
from torchgpipe_amd.stream import AbstractStream, get_device

__all__: List[str] = []


class Portal:
    __slots__ = ('tensor', 'tensor_life', 'grad')

    def __init__(self, tensor: Optional[Tensor], tensor_life: int) -> None:
        self.tensor: Optional[Tensor] = None
        self.tensor_life = 0
        self.put_tensor(tensor, tensor_life)
        self.grad: Optional[Tensor] = None

    def blue(self) -> Tensor:
        tensor = self.use_tensor()
        if tensor is None:
            return get_phony(torch.device('cpu'), requires_grad=False)
        return PortalBlue.apply(self, tensor)

    def orange(self, phony: Tensor) -> Optional[Tensor]:
        self.check_tensor_life()
        if self.tensor is None:
            return self.use_tensor()
        return PortalOrange.apply(self, phony)

    def copy(self, prev_stream: AbstractStream, next_stream: AbstractStream,
             phony: Tensor) -> Tensor:
        if self.tensor is None:
            return get_phony(torch.device('cpu'), requires_grad=False)
        return PortalCopy.apply(self, prev_stream, next_stream, phony)

    def check_tensor_life(self) -> None:
        if self.tensor_life <= 0:
            raise RuntimeError('tensor in portal has been removed')

    def put_tensor(self, tensor: Optional[Tensor], tensor_life: int) -> None:
        self.tensor_life = tensor_life
        self.tensor = tensor if tensor_life > 0 else None

    def use_tensor(self) -> Optional[Tensor]:
        self.check_tensor_life()
        tensor = self.tensor
        self.tensor_life -= 1
        if self.tensor_life <= 0:
            self.tensor = None
        return tensor

    def put_grad(self, grad: Tensor) -> None:
        self.grad = grad

    def use_grad(self) -> Tensor:
        if self.grad is None:
            raise RuntimeError('grad in portal has been removed or never set')
        grad, self.grad = self.grad, None
        return grad


class PortalBlue(torch.autograd.Function):
    @staticmethod
    def forward(ctx, portal: Portal, tensor: Tensor) -> Tensor:  # type: ignore[override]
        ctx.portal = portal
        return get_phony(tensor.device, requires_grad=False).detach()

    @staticmethod
    def backward(ctx, grad_phony: Tensor) -> Tuple[None, Tensor]:  # type: ignore[override]
        return None, ctx.portal.use_grad()


class PortalOrange(torch.autograd.Function):
    @staticmethod
    def forward(ctx, portal: Portal, phony: Tensor) -> Tensor:  # type: ignore[override]
        ctx.portal = portal
        tensor = portal.use_tensor()
        assert tensor is not None
        return tensor.detach()

    @staticmethod
    def backward(ctx, grad: Tensor) -> Tuple[None, None]:  # type: ignore[override]
        ctx.portal.put_grad(grad)
        return None, None


class PortalCopy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, portal: Portal, prev_stream: AbstractStream,  # type: ignore[override]
                next_stream: AbstractStream, phony: Tensor) -> Tensor:
        ctx.portal = portal
        assert portal.tensor is not None
        portal.tensor, = Copy.forward(ctx, prev_stream, next_stream, portal.tensor)
        return get_phony(get_device(next_stream), requires_grad=False).detach()

    @staticmethod
    def backward(ctx, grad_phony: Tensor) -> Tuple[None, None, None, None]:  # type: ignore[override]
        portal = ctx.portal
        assert portal.grad is not None
        _, _, portal.grad = Copy.backward(ctx, portal.grad)
        return None, None, None, None
