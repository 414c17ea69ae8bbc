"""Stream-aware device-to-device hand-off (``Copy``) and stream fences (``Wait``).

Parity: ``torchgpipe/copy.py:25-107``.

``Copy`` moves every tensor of a micro-batch from partition ``j-1``'s device
to partition ``j``'s device.  The copy is enqueued on the *destination*
side copy stream (under both the source and destination copy streams as
current streams), so on a multi-GPU MI355X node it becomes a
``hipMemcpyPeerAsync`` over the direct xGMI link between the two GPUs and
overlaps with compute on both sides.  The allocator is told about the
cross-stream lifetimes with ``record_stream`` on both ends.  Backward copies
the gradients in the reverse direction on the same stream pair.

``Wait`` is a value identity that inserts a stream→stream dependency
(HIP event record + wait): forward makes ``next`` wait for ``prev``;
backward makes ``prev`` wait for ``next``.
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from torchgpipe_amd.stream import (AbstractStream, current_stream, get_device, record_stream,
                                   use_stream, wait_stream)

__all__: List[str] = []

Tensors = Tuple[Tensor, ...]


def _transfer(tensors: Tensors,
              src_stream: AbstractStream,
              dst_stream: AbstractStream,
              device: torch.device,
              consumer_stream: AbstractStream) -> List[Tensor]:
    out: List[Tensor] = []
    with use_stream(src_stream), use_stream(dst_stream):
        for x in tensors:
            # Peer (GPU→GPU) copies are stream-ordered; anything touching the
            # host must stay blocking because CPU "streams" carry no ordering.
            y = x.to(device, non_blocking=x.is_cuda and device.type == 'cuda')
            out.append(y)
            # x is read on the copy stream, not the stream it was allocated on.
            record_stream(x, src_stream)
            # y is allocated on the copy stream and consumed on the compute stream.
            record_stream(y, consumer_stream)
    return out


class Copy(torch.autograd.Function):
    """Copy tensors between devices on explicit streams."""

    @staticmethod
    def forward(ctx, prev_stream: AbstractStream,  # type: ignore[override]
                next_stream: AbstractStream, *input: Tensor) -> Tensors:
        ctx.prev_stream = prev_stream
        ctx.next_stream = next_stream
        dst = get_device(next_stream)
        return tuple(_transfer(input, prev_stream, next_stream, dst, current_stream(dst)))

    @staticmethod
    def backward(ctx, *grad_output: Tensor) -> Tuple[Optional[Tensor], ...]:  # type: ignore[override]
        prev_stream = ctx.prev_stream
        next_stream = ctx.next_stream
        src = get_device(prev_stream)
        grads = _transfer(grad_output, next_stream, prev_stream, src, current_stream(src))
        return (None, None) + tuple(grads)


class Wait(torch.autograd.Function):
    """Fence: ``next_stream`` waits for ``prev_stream`` (reverse in backward)."""

    @staticmethod
    def forward(ctx, prev_stream: AbstractStream,  # type: ignore[override]
                next_stream: AbstractStream, *input: Tensor) -> Tensors:
        ctx.prev_stream = prev_stream
        ctx.next_stream = next_stream
        wait_stream(next_stream, prev_stream)
        return tuple(x.detach() for x in input)

    @staticmethod
    def backward(ctx, *grad_input: Tensor) -> Tuple[Optional[Tensor], ...]:  # type: ignore[override]
        wait_stream(ctx.prev_stream, ctx.next_stream)
        return (None, None) + grad_input
