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

A multi-tensor hop between two GPUs (AmoebaNet's ``(x, skip)`` boundaries,
their gradients, several skips bound for one partition) is *packed*: the HIP
segment-copy kernel (``copy_segments``) gathers the tensors into one byte
buffer on the source GPU, one peer copy moves it over xGMI, and the
destination tensors are zero-copy views into the received buffer -- one DMA
per hop instead of one per tensor.

``Wait`` is a value identity that inserts a stream→stream dependency
(HIP event record + wait): forward makes ``next`` wait for ``prev``;
backward makes ``prev`` wait for ``next``.
"""
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from torchgpipe_amd.stream import (AbstractStream, current_stream, get_device, record_stream,
                                   use_stream, wait_stream)

Tensors = Tuple[Tensor, ...]

# counters of packed hops (tests / diagnostics)
packed_hops = 0

# Skip hops (PortalCopy) pack only tensors below this size: every packed tensor is a view
# of one received buffer, so the buffer -- all of the route's skips -- would stay alive
# until the last of them is popped, while a separately copied skip is freed as soon as its
# pop partition is done with it (tensor-life accounting, skip/portal.py).  Above a few MiB
# a copy's launch cost is noise next to its transfer, so packing them saves nothing.
SKIP_PACK_MAX_BYTES = 4 << 20


def _packable(tensors: Tensors, device: torch.device) -> bool:
    if len(tensors) < 2 or device.type != 'cuda':
        return False
    src = tensors[0].device
    return (src.type == 'cuda' and src != device
            and all(t.device == src and not t.is_sparse for t in tensors))


def _packed_transfer(tensors: Tensors, device: torch.device) -> List[Tensor]:
    """Pack on the source GPU, one peer copy, views on the destination (current streams)."""
    global packed_hops
    from torchgpipe_amd.ops import misc
    nbytes = misc.packed_nbytes(tensors)
    buf = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=tensors[0].device)
    misc.pack([t.detach() for t in tensors], buf)
    moved = buf.to(device, non_blocking=True)
    out: List[Tensor] = []
    pos = 0
    for t in tensors:
        size = t.numel() * t.element_size()
        out.append(moved[pos:pos + size].view(t.dtype).view(t.shape))
        pos = (pos + size + 15) // 16 * 16
    packed_hops += 1
    return out

__all__: List[str] = []


def _transfer(tensors: Tensors,
              src_stream: AbstractStream,
              dst_stream: AbstractStream,
              device: torch.device,
              consumer_stream: AbstractStream,
              pack_max: Optional[int] = None) -> List[Tensor]:
    """Move ``tensors`` to ``device``; several GPU tensors go as one packed hop (only those
    below ``pack_max`` bytes when given, the others one by one)."""
    if pack_max is not None:
        small = [k for k, t in enumerate(tensors) if t.numel() * t.element_size() < pack_max]
        if len(small) < len(tensors):
            moved: List[Optional[Tensor]] = [None] * len(tensors)
            if len(small) >= 2:
                for k, y in zip(small, _transfer(tuple(tensors[k] for k in small), src_stream,
                                                 dst_stream, device, consumer_stream)):
                    moved[k] = y
            rest = [k for k in range(len(tensors)) if moved[k] is None]
            for k in rest:
                moved[k] = _transfer((tensors[k],), src_stream, dst_stream, device,
                                     consumer_stream)[0]
            return [t for t in moved if t is not None]
    out: List[Tensor] = []
    with use_stream(src_stream), use_stream(dst_stream):
        if _packable(tensors, device):
            out = _packed_transfer(tensors, device)
            for x in tensors:
                record_stream(x, src_stream)
            for y in out:
                record_stream(y, consumer_stream)
            return out
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
        return tuple(_transfer(input, prev_stream, next_stream, dst, current_stream(dst),
                               getattr(ctx, 'pack_max', None)))

    @staticmethod
    def backward(ctx, *grad_output: Tensor) -> Tuple[Optional[Tensor], ...]:  # type: ignore[override]
        prev_stream = ctx.prev_stream
        next_stream = ctx.next_stream
        src = get_device(prev_stream)
        grads = _transfer(grad_output, next_stream, prev_stream, src, current_stream(src),
                          getattr(ctx, 'pack_max', None))
        return (None, None) + tuple(grads)


class Wait(torch.autograd.Function):
    """Fence: ``next_stream`` waits for ``prev_stream`` (reverse in backward)."""

    @staticmethod
    def forward(ctx, prev_stream: AbstractStream,  # type: ignore[override]
                next_stream: AbstractStream, *input: Tensor) -> Tensors:
        ctx.prev_stream = prev_stream
        ctx.next_stream = next_stream
        wait_stream(next_stream, prev_stream)
        # the consumer may be a lane (GPipe(overlap_forward=True)) rather than the stream the
        # tensors were allocated on: keep their blocks from the allocator until it is done
        for x in input:
            record_stream(x, next_stream)
        return tuple(x.detach() for x in input)

    @staticmethod
    def backward(ctx, *grad_input: Tensor) -> Tuple[Optional[Tensor], ...]:  # type: ignore[override]
        wait_stream(ctx.prev_stream, ctx.next_stream)
        for g in grad_input:
            if g is not None:
                record_stream(g, ctx.prev_stream)
        return (None, None) + grad_input
