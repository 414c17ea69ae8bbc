"""Micro-batch data model (layer L3): ``Batch``, ``check``, ``scatter``, ``gather``.

Parity: ``torchgpipe/microbatch.py:17-177``.  A ``Batch`` is either *atomic*
(a single tensor) or a tuple of tensors, with in-place item/slice assignment
so that autograd wrappers (Copy, Wait, Fork/Join, portals) can replace the
tensors of a micro-batch without re-wrapping.

``scatter`` returns views (``Tensor.chunk``), as in the reference, so the
number of micro-batches may be smaller than ``chunks`` (N=6, chunks=4 → 3).
"""
import typing
from typing import Callable, Iterator, List, Tuple, Union, cast

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
