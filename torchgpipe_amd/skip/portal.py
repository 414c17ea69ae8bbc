"""Portals: carry a skip tensor outside the autograd graph.

Reference behaviour: ``torchgpipe/skip/portal.py:22-227``.  A skip tensor stashed in
partition ``j`` and popped in ``k`` would, if passed through the pipeline as a regular
tensor, be copied through every intermediate partition and kept alive there.  A portal
instead *hides* it behind three autograd functions tied to the micro-batch lane by
phonies:

* ``PortalBlue`` (stash side) consumes the tensor and returns a phony that is joined
  into the lane; its backward emits the gradient that the pop side deposited.
* ``PortalCopy`` moves hidden tensors directly from ``j``'s device to ``k``'s (one
  xGMI hop on the copy streams) and their gradients back.  Unlike the reference, which
  copies each skip on its own (``torchgpipe/skip/portal.py:199-227``), one
  ``PortalCopy`` carries *every* skip of a micro-batch on the same (source,
  destination) route: ``Copy`` packs them into one buffer with the HIP segment-copy
  kernel, so U-Net's long skips into one partition cost one peer DMA per micro-batch,
  not one per skip.
* ``PortalOrange`` (pop side) returns the hidden tensor; its backward stores the
  incoming gradient into the portal.

Tensor life.  A portal frees its tensor as soon as the last user has run.  Users are
the ``blue()``, ``orange()`` and recomputed ``blue()`` / ``orange()`` calls; which of
them exist depends on whether the cell is checkpointed:

=============================  ====================  ==================
call                           checkpointed (life 3)  plain (life 2)
=============================  ====================  ==================
``blue()`` (stash)             3 → 2                  2 → 1
``copy()``                     keeps the life         keeps the life
``orange()`` (pop)             2 → 1                  1 → 0, freed
``orange()`` recomputed        1 → 0, freed           --
``blue()`` recomputed          re-put with life 1,    --
                               1 → 0, freed
=============================  ====================  ==================
"""
from typing import List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from torchgpipe_amd.copy import SKIP_PACK_MAX_BYTES, Copy
from torchgpipe_amd.phony import get_phony
from torchgpipe_amd.stream import AbstractStream, get_device

__all__: List[str] = []

# number of PortalCopy hops issued (one per route and micro-batch; tests / diagnostics)
portal_hops = 0


class Portal:
    """Holds one skip tensor (with a use count) and, later, its gradient."""

    __slots__ = ('tensor', 'tensor_life', 'grad')

    def __init__(self, tensor: Optional[Tensor], tensor_life: int) -> None:
        self.tensor: Optional[Tensor] = None
        self.tensor_life = 0
        self.grad: Optional[Tensor] = None
        self.put_tensor(tensor, tensor_life)

    # -- the three faces --------------------------------------------------------------------

    def blue(self) -> Tensor:
        """Stash side: hide the tensor, return the phony to join into the lane."""
        tensor = self.use_tensor()
        if tensor is None:
            return get_phony(torch.device('cpu'), requires_grad=False)
        return PortalBlue.apply(self, tensor)

    def orange(self, phony: Tensor) -> Optional[Tensor]:
        """Pop side: the hidden tensor, as a fresh autograd leaf of the lane."""
        self.check_tensor_life()
        if self.tensor is None:
            return self.use_tensor()
        return PortalOrange.apply(self, phony)

    def copy(self, prev_stream: AbstractStream, next_stream: AbstractStream,
             phony: Tensor) -> Tensor:
        """Move the hidden tensor to ``next_stream``'s device (see :func:`copy_portals`)."""
        return copy_portals([self], prev_stream, next_stream, phony)

    # -- bookkeeping ------------------------------------------------------------------------

    def check_tensor_life(self) -> None:
        if self.tensor_life <= 0:
            raise RuntimeError('tensor in portal has been removed')

    def put_tensor(self, tensor: Optional[Tensor], tensor_life: int) -> None:
        self.tensor_life = tensor_life
        self.tensor = tensor if tensor_life > 0 else None

    def use_tensor(self) -> Optional[Tensor]:
        """Take the tensor, spending one life; the last use drops the reference."""
        self.check_tensor_life()
        tensor = self.tensor
        self.tensor_life -= 1
        if self.tensor_life <= 0:
            self.tensor = None
        return tensor

    def put_grad(self, grad: Tensor) -> None:
        self.grad = grad

    def use_grad(self) -> Tensor:
        """Take the gradient (once)."""
        grad = self.grad
        if grad is None:
            raise RuntimeError('grad in portal has been removed or never set')
        self.grad = None
        return grad


def copy_portals(portals: Sequence[Portal], prev_stream: AbstractStream,
                 next_stream: AbstractStream, phony: Tensor) -> Tensor:
    """Move the tensors of ``portals`` (all stashed on ``prev_stream``'s device) to
    ``next_stream``'s device as ONE hop, and their gradients back in backward.

    Returns the phony to join into the micro-batch lane (a CPU phony if no portal holds
    a tensor, e.g. ``stash(name, None)``).
    """
    global portal_hops
    live = tuple(p for p in portals if p.tensor is not None)
    if not live:
        return get_phony(torch.device('cpu'), requires_grad=False)
    portal_hops += 1
    return PortalCopy.apply(live, prev_stream, next_stream, phony)


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
    """The hidden tensors of several portals on one route, moved as one (packed) hop."""

    @staticmethod
    def forward(ctx, portals: Tuple[Portal, ...], prev_stream: AbstractStream,  # type: ignore[override]
                next_stream: AbstractStream, phony: Tensor) -> Tensor:
        ctx.portals = portals
        # large skips travel (and are freed) one by one, small ones packed (copy.py)
        ctx.pack_max = SKIP_PACK_MAX_BYTES
        moved = Copy.forward(ctx, prev_stream, next_stream,
                             *[p.tensor for p in portals])  # type: ignore[misc]
        for portal, tensor in zip(portals, moved):
            portal.tensor = tensor
        return get_phony(get_device(next_stream), requires_grad=False).detach()

    @staticmethod
    def backward(ctx, grad_phony: Tensor) -> Tuple[None, None, None, None]:  # type: ignore[override]
        portals = ctx.portals
        grads = [p.grad for p in portals]
        assert all(g is not None for g in grads)
        moved = Copy.backward(ctx, *grads)[2:]  # type: ignore[arg-type]
        for portal, grad in zip(portals, moved):
            portal.grad = grad
        return None, None, None, None
