"""Activation checkpointing with *preceding* recomputation.

Parity: ``torchgpipe/checkpoint.py:1-308``.  ``torch.utils.checkpoint`` fuses
"recompute" and "backprop through the recomputed graph" into one autograd
node, so recomputation can only start once the output gradient has arrived.
In a pipeline that wastes the time the gradient spends crossing the xGMI
link.  As in the reference, checkpointing is split into two autograd nodes
that share a one-slot mailbox:

* ``Checkpoint`` — forward runs the partition under ``no_grad``; backward
  back-propagates through the graph that ``Recompute`` built.
* ``Recompute`` — a phony-valued node placed (via Fork/Join) *before* the
  ``Wait`` that guards the gradient copy, so the autograd engine runs the
  recomputation while the gradient is still in flight.

Multi-process schedules (``torchgpipe_amd.parallel``) drive the same pair
explicitly: ``Checkpointing.recompute_now()`` is issued right after the
receive for the output gradient has been posted, and ``Checkpoint.backward``
then finds the recomputed graph already waiting in the mailbox.

RNG replay (K4 in SURVEY §2.4).  Two mechanisms, both deterministic:

1. PyTorch-managed randomness (``nn.Dropout`` …): the CPU and device
   generator states are snapshotted at checkpoint time and restored inside
   ``torch.random.fork_rng`` during recomputation (reference behaviour).
2. Framework HIP RNG ops (``torchgpipe_amd.ops.dropout`` – Philox4x32-10 with
   explicit ``(seed, offset)``): an ``RngTape`` records every ``(seed,
   offset)`` pair drawn while checkpointing and replays exactly those pairs
   during recomputation, without reading or mutating any generator from the
   autograd thread.
"""
from collections import deque
from contextlib import contextmanager
import threading
from typing import Any, Deque, Generator, Optional, Tuple, Union

import torch
from torch import Tensor

from torchgpipe_amd.dependency import fork, join
from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.phony import get_phony
from torchgpipe_amd.utils.rng import RngTape

__all__ = ['is_checkpointing', 'is_recomputing', 'checkpoint', 'Checkpointing']

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]
Recomputed = Tuple[TensorOrTensors, Tensors]  # (output, input_leaf)


class _Flags(threading.local):
    def __init__(self) -> None:
        self.is_checkpointing = False
        self.is_recomputing = False


_flags = _Flags()


@contextmanager
def enable_checkpointing() -> Generator[None, None, None]:
    prev = _flags.is_checkpointing
    _flags.is_checkpointing = True
    try:
        yield
    finally:
        _flags.is_checkpointing = prev


@contextmanager
def enable_recomputing() -> Generator[None, None, None]:
    prev = _flags.is_recomputing
    _flags.is_recomputing = True
    try:
        yield
    finally:
        _flags.is_recomputing = prev


def is_checkpointing() -> bool:
    """True while the current thread runs a forward pass under checkpointing."""
    return _flags.is_checkpointing


def is_recomputing() -> bool:
    """True while the current thread re-runs a forward pass for backprop.

    Use it to avoid duplicated side effects (counters, running statistics)::

        def forward(self, x):
            if not is_recomputing():
                self.counter += 1
            return x
    """
    return _flags.is_recomputing


class RNGSnapshot:
    """CPU + device generator state captured at checkpoint time."""

    __slots__ = ('device', 'cpu_state', 'gpu_state')

    def __init__(self, device: torch.device) -> None:
        self.device = device
        self.cpu_state = torch.get_rng_state()
        self.gpu_state: Optional[Tensor] = None
        # Inside a hipGraph capture (parallel/graph.py, RNG-free partitions only) the
        # device generator state can be neither read nor restored: skip it.
        if device.type == 'cuda' and not torch.cuda.is_current_stream_capturing():
            self.gpu_state = torch.cuda.get_rng_state(device)

    @contextmanager
    def restored(self) -> Generator[None, None, None]:
        devices = [self.device] if self.gpu_state is not None else []
        with torch.random.fork_rng(devices):
            torch.set_rng_state(self.cpu_state)
            if self.gpu_state is not None:
                torch.cuda.set_rng_state(self.gpu_state, self.device)
            yield


class _Shared:
    """State shared by one Checkpoint/Recompute pair (the reference uses deques)."""

    __slots__ = ('function', 'input_atomic', 'recomputed', 'rng', 'tape', 'inputs',
                 'versions')

    def __init__(self, function: Any, input_atomic: bool) -> None:
        self.function = function
        self.input_atomic = input_atomic
        # the Checkpoint node's inputs, for a recomputation its backward has to run itself;
        # held here rather than in the node's saved tensors so a pipeline that recomputes
        # ahead and back-propagates through the recomputed graph can release them while a
        # loss still references the node (PipelineStage's last stage)
        self.inputs: Optional[Tensors] = None
        # the inputs' version counters at the checkpointed forward: with the inputs held
        # here instead of in saved tensors, autograd's own check is gone, so the
        # recomputation checks them itself (an in-place change in between would recompute
        # from the changed value and give wrong gradients silently)
        self.versions: Optional[Tuple[int, ...]] = None
        self.recomputed: Deque[Recomputed] = deque(maxlen=1)
        self.rng: Deque[RNGSnapshot] = deque(maxlen=1)
        self.tape = RngTape()

    def run_recompute(self, inputs: Tensors) -> None:
        if self.versions is not None and \
                tuple(x._version for x in inputs) != self.versions:
            raise RuntimeError('one of the inputs of a checkpointed micro-batch has been '
                               'modified by an inplace operation before its recomputation '
                               f'(versions {self.versions} at the forward, '
                               f'{tuple(x._version for x in inputs)} now)')
        leaves = tuple(x.detach().requires_grad_(x.requires_grad) for x in inputs)
        snapshot = self.rng.pop()
        with snapshot.restored(), self.tape.replaying():
            with torch.enable_grad(), enable_recomputing():
                output = self.function(leaves[0] if self.input_atomic else leaves)
        self.recomputed.append((output, leaves))


class Checkpoint(torch.autograd.Function):
    @staticmethod
    def forward(ctx, phony: Tensor, shared: _Shared,  # type: ignore[override]
                *input: Tensor) -> TensorOrTensors:
        ctx.shared = shared
        shared.inputs = input
        shared.rng.append(RNGSnapshot(input[0].device))
        with torch.no_grad(), enable_checkpointing(), shared.tape.recording():
            output = shared.function(input[0] if shared.input_atomic else input)
        # (after the function: its own in-place ops on its inputs are the recomputation's
        # business, as in the reference; what must not happen is a change in between)
        shared.versions = tuple(x._version for x in input)
        return output

    @staticmethod
    def backward(ctx, *grad_output: Tensor) -> Tuple[Optional[Tensor], ...]:  # type: ignore[override]
        shared: _Shared = ctx.shared
        if not shared.recomputed:
            # Nobody scheduled the recomputation ahead of time: do it now.
            assert shared.inputs is not None, 'checkpoint inputs already released'
            shared.run_recompute(shared.inputs)
        shared.inputs = None
        output, leaves = shared.recomputed.pop()
        outputs = output if isinstance(output, tuple) else (output,)
        pairs = [(y, g) for y, g in zip(outputs, grad_output) if y.requires_grad]
        if pairs:
            torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
        return (None, None) + tuple(x.grad for x in leaves)


class Recompute(torch.autograd.Function):
    @staticmethod
    def forward(ctx, phony: Tensor, shared: _Shared,  # type: ignore[override]
                *input: Tensor) -> Tensor:
        ctx.shared = shared
        ctx.save_for_backward(*input)
        return phony

    @staticmethod
    def backward(ctx, *grad_output: Tensor) -> Tuple[None, ...]:  # type: ignore[override]
        ctx.shared.run_recompute(ctx.saved_tensors)
        return (None, None) + tuple(None for _ in ctx.saved_tensors)


class Checkpointing:
    """Build a ``Checkpoint``/``Recompute`` pair around ``function(batch)``."""

    def __init__(self, function: Any, batch: Batch) -> None:
        self.function = function
        self.batch = batch
        self.shared = _Shared(function, batch.atomic)

    def checkpoint(self) -> Batch:
        """Run the forward pass without keeping activations."""
        # A grad-requiring phony guarantees that the Checkpoint node is part of
        # the graph even when no input requires grad.
        phony = get_phony(self.batch[0].device, requires_grad=True)
        output = Checkpoint.apply(phony, self.shared, *tuple(self.batch))
        return Batch(output)

    def recompute(self, batch: Batch) -> None:
        """Attach a ``Recompute`` node ahead of ``batch`` (autograd-driven)."""
        batch[0], phony = fork(batch[0])
        phony = Recompute.apply(phony, self.shared, *tuple(self.batch))
        batch[0] = join(batch[0], phony)

    def recompute_now(self) -> None:
        """Recompute eagerly (explicitly scheduled pipelines)."""
        if not self.shared.recomputed:
            self.shared.run_recompute(tuple(self.batch))

    def take_recomputed(self) -> Tuple[Tuple[Tensor, ...], Tuple[Tensor, ...]]:
        """The recomputation's ``(outputs, input leaves)``, for a caller that back-propagates
        through the recomputed graph itself (``PipelineStage``: one backward call per
        micro-batch instead of the Checkpoint node's reentrant one); the Checkpoint node
        then never runs."""
        output, leaves = self.shared.recomputed.pop()
        self.shared.inputs = None  # the Checkpoint node will not run
        return (output if isinstance(output, tuple) else (output,)), leaves


def checkpoint(function: Any, input: TensorOrTensors) -> TensorOrTensors:
    """Drop-in ``torch.utils.checkpoint``-like helper (tests / debugging)."""
    batch = Batch(input)
    chk = Checkpointing(function, batch)
    out = chk.checkpoint()
    chk.recompute(out)
    return out.tensor_or_tensors


def save_rng_states(device: torch.device, rng_states: Deque[RNGSnapshot]) -> None:
    rng_states.append(RNGSnapshot(device))


@contextmanager
def restore_rng_states(device: torch.device,
                       rng_states: Deque[RNGSnapshot]) -> Generator[None, None, None]:
    with rng_states.pop().restored():
        yield
