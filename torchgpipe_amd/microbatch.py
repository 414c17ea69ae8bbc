"""Micro-batch data model (layer L3): ``Batch``, ``check``, ``scatter``, ``gather``.

Parity: ``torchgpipe/microbatch.py:17-177``.  A ``Batch`` is either *atomic*
(a single tensor) or a tuple of tensors, with in-place item/slice assignment
so that autograd wrappers (Copy, Wait, Fork/Join, portals) can replace the
tensors of a micro-batch without re-wrapping.

``scatter`` returns views (``Tensor.chunk``), as in the reference, so the
number of micro-batches may be smaller than ``chunks`` (N=6, chunks=4 → 3).
"""
import typing
from typing import Callable, Iterator, List, Optional, Sequence, Tuple, Union, cast

import torch
from torch import Tensor

__all__: List[str] = []

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]
Function = Callable[[TensorOrTensors], TensorOrTensors]


class Batch:
    """An atomic tensor or a tuple of tensors travelling through the pipeline."""

    __slots__ = ('value', 'atomic')

    def __init__(self, value: TensorOrTensors) -> None:
        self.value = value
        self.atomic = torch.is_tensor(value)

    @property
    def tensor(self) -> Tensor:
        if not self.atomic:
            raise AttributeError('not atomic batch')
        return cast(Tensor, self.value)

    @property
    def tensors(self) -> Tensors:
        if self.atomic:
            raise AttributeError('batch is atomic')
        return cast(Tensors, self.value)

    @property
    def tensor_or_tensors(self) -> TensorOrTensors:
        return self.value

    def call(self, function: Function) -> 'Batch':
        return Batch(function(self.value))

    def __repr__(self) -> str:
        return f'Batch[atomic={self.atomic!r}]({self.value!r})'

    def __iter__(self) -> Iterator[Tensor]:
        if self.atomic:
            yield cast(Tensor, self.value)
        else:
            yield from cast(Tensors, self.value)

    def __len__(self) -> int:
        return 1 if self.atomic else len(cast(Tensors, self.value))

    def __getitem__(self, index: int) -> Tensor:
        if not self.atomic:
            return cast(Tensors, self.value)[index]
        if index != 0:
            raise IndexError('atomic batch allows index 0 only')
        return cast(Tensor, self.value)

    @typing.overload
    def __setitem__(self, index: int, value: Tensor) -> None: ...

    @typing.overload
    def __setitem__(self, index: slice, value: Tensors) -> None: ...

    def __setitem__(self, index, value) -> None:  # type: ignore[no-untyped-def]
        if isinstance(index, slice):
            if not (index.start is None and index.stop is None and index.step is None):
                raise NotImplementedError('only slice [:] supported')
            if self.atomic:
                if len(value) != 1:
                    raise IndexError('atomic batch cannot be replaced with multiple tensors')
                self.value = value[0]
            else:
                self.value = tuple(value)
            return

        if self.atomic:
            if index != 0:
                raise IndexError('atomic batch allows index 0 only')
            self.value = value
            return

        values = list(cast(Tensors, self.value))
        values[index] = value
        self.value = tuple(values)


def check(input: TensorOrTensors) -> None:
    """Raise ``TypeError`` unless ``input`` is a tensor or (nested) tuple of tensors."""
    if isinstance(input, tuple):
        for x in input:
            check(x)
        return
    if not isinstance(input, Tensor):
        raise TypeError(f'expected Tensor, but got {input.__class__.__name__}')


def scatter(input: TensorOrTensors, chunks: int) -> List[Batch]:
    """Split a mini-batch along dim 0 into at most ``chunks`` micro-batches (views)."""
    if isinstance(input, Tensor):
        return [Batch(x) for x in input.chunk(chunks)]
    per_tensor = [t.chunk(chunks) for t in input]
    counts = {len(c) for c in per_tensor}
    if len(counts) > 1:
        # Mirror zip() truncation of the reference: shortest chunk list wins.
        n = min(counts)
        per_tensor = [c[:n] for c in per_tensor]
    return [Batch(tuple(parts)) for parts in zip(*per_tensor)]


def gather(outputs: List[Batch]) -> TensorOrTensors:
    """Concatenate micro-batch outputs back into a mini-batch."""
    if outputs[0].atomic:
        return torch.cat(tuple(b.tensor for b in outputs))
    columns = zip(*(b.tensors for b in outputs))
    return tuple(torch.cat(col) for col in columns)


class _GatherInto(torch.autograd.Function):
    """Autograd view of buffers that already hold every micro-batch's output.

    Forward returns the buffers (filled by :class:`Gatherer` while the pipeline ran);
    backward hands each micro-batch output its slice of the gradient -- views, no copy
    (the reference's ``torch.cat`` backward also slices).
    """

    @staticmethod
    def forward(ctx, bounds: List[Tuple[int, int]], nbuf: int,  # type: ignore[override]
                *tensors: Tensor) -> Tensors:
        ctx.bounds = bounds
        ctx.nbuf = nbuf
        return tuple(b.detach() for b in tensors[:nbuf])

    @staticmethod
    def backward(ctx, *grads: Tensor):  # type: ignore[override]
        out: List[Optional[Tensor]] = [None, None] + [None] * ctx.nbuf
        for lo, hi in ctx.bounds:
            for g in grads:
                out.append(None if g is None else g[lo:hi])
        return tuple(out)


class Gatherer:
    """K11 zero-copy gather: micro-batch outputs land in preallocated mini-batch buffers.

    ``put(i, batch)`` runs when micro-batch ``i`` leaves the last partition: its tensors
    are copied into their slice of the output buffers on a side stream (overlapping the
    remaining micro-batches' compute) instead of one ``torch.cat`` after the pipeline;
    :meth:`result` fences the side streams and returns the buffers through
    :class:`_GatherInto`.  Falls back to :func:`gather` when an output's first
    dimension is not its micro-batch size, or on CPU.
    """

    def __init__(self, sizes: Sequence[int], streams: Optional[Sequence[object]] = None) -> None:
        self.sizes = list(sizes)
        self.bounds: List[Tuple[int, int]] = []
        pos = 0
        for n in self.sizes:
            self.bounds.append((pos, pos + n))
            pos += n
        self.total = pos
        self.streams = streams
        self.buffers: Optional[List[Tensor]] = None
        self.atomic = True
        self.ok = True
        self.used: List[object] = []

    def put(self, i: int, batch: Batch, stream: Optional[object] = None) -> None:
        """Copy micro-batch ``i``'s outputs into their slice, after ``stream`` (the stream
        that computed them; default: the device's current stream)."""
        from torchgpipe_amd.stream import current_stream, record_stream, use_stream, wait_stream
        if not self.ok:
            return
        tensors = list(batch)
        if self.buffers is None:
            self.atomic = batch.atomic
            if any(not isinstance(t, Tensor) or not t.is_cuda or t.dim() == 0
                   for t in tensors):
                self.ok = False
                return
            self.buffers = [torch.empty((self.total, *t.shape[1:]), dtype=t.dtype,
                                        device=t.device) for t in tensors]
        lo, hi = self.bounds[i]
        if len(tensors) != len(self.buffers) or any(not isinstance(t, Tensor) for t in tensors) \
                or any(
                t.shape[0] != hi - lo or t.shape[1:] != b.shape[1:] or t.dtype != b.dtype
                or t.device != b.device for t, b in zip(tensors, self.buffers)):
            self.ok = False
            return
        compute = stream if stream is not None else current_stream(tensors[0].device)
        side = self.streams[i] if self.streams is not None else compute
        wait_stream(side, compute)  # type: ignore[arg-type]
        with use_stream(side):  # type: ignore[arg-type]
            for t, b in zip(tensors, self.buffers):
                b[lo:hi].copy_(t.detach(), non_blocking=True)
                record_stream(t, side)  # type: ignore[arg-type]
                # the buffers were allocated on the compute stream: keep them alive until
                # the side stream's copies are done, even if result() falls back
                record_stream(b, side)  # type: ignore[arg-type]
        self.used.append(side)

    def result(self, outputs: List[Batch]) -> TensorOrTensors:
        from torchgpipe_amd.stream import current_stream, wait_stream
        if self.buffers is not None:
            # fence the side-stream copies on both return paths (a later micro-batch may
            # have failed the shape check after earlier ones were already queued)
            compute = current_stream(self.buffers[0].device)
            seen = set()
            for side in self.used:
                if id(side) not in seen:
                    seen.add(id(side))
                    wait_stream(compute, side)  # type: ignore[arg-type]
        if not self.ok or self.buffers is None:
            return gather(outputs)
        flat = [t for b in outputs for t in b]
        out = _GatherInto.apply(self.bounds, len(self.buffers), *self.buffers, *flat)
        return out[0] if self.atomic else tuple(out)
