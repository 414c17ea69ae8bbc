"""Deterministic Philox ``(seed, offset)`` management for framework RNG ops.

The reference replays dropout during recomputation by snapshotting and
restoring the *global* generators (``torchgpipe/checkpoint.py:191-231``),
which mutates process-global state from autograd worker threads.

Framework RNG ops (the HIP dropout kernels in ``torchgpipe_amd.ops``) instead
take an explicit Philox4x32-10 ``(seed, offset)`` pair per call.  Pairs are
reserved from the device's default generator (advancing its offset exactly
like a PyTorch RNG op would), and an :class:`RngTape` attached to a
checkpointed cell records the pairs drawn while checkpointing and hands back
the very same pairs during recomputation.  Replay therefore touches no
generator at all and is bit-exact by construction.

Because the pair is explicit, backward kernels regenerate the dropout mask
from ``(seed, offset)`` instead of storing it — no mask tensor is kept alive.

Captured cells (:mod:`torchgpipe_amd.parallel.segments`) cannot use host-side pairs: a
graph replay would re-issue the captured constants and draw the same mask every step.
Inside a :func:`slot_scope` the RNG ops instead read a *device-resident* state
(:class:`PhiloxSlot`, int64 ``[seed, base offset]``) when their kernel runs, and the
host-side offset they pass is the counter position *within the cell*.  The pipeline
writes fresh ``(seed, base offset)`` values (reserved from the device generator) into the
slot before each replay; the forward and the recomputation of a cell read the same slot,
so their masks agree bit for bit.
"""
from contextlib import contextmanager
import threading
from typing import Generator, List, Optional, Tuple

import torch

__all__ = ['RngTape', 'philox_pair', 'current_tape', 'PhiloxSlot', 'slot_scope', 'philox_draw',
           'reserve']

SeedOffset = Tuple[int, int]


class _TapeState(threading.local):
    def __init__(self) -> None:
        self.tape: Optional['RngTape'] = None
        self.slot: Optional['PhiloxSlot'] = None


_state = _TapeState()
_gen_lock = threading.Lock()


class RngTape:
    """Records (while checkpointing) and replays (while recomputing) Philox pairs."""

    __slots__ = ('entries', 'cursor', 'mode')

    def __init__(self) -> None:
        self.entries: List[SeedOffset] = []
        self.cursor = 0
        self.mode: Optional[str] = None

    @contextmanager
    def _activate(self, mode: str) -> Generator[None, None, None]:
        prev = _state.tape
        prev_mode = self.mode
        self.mode = mode
        _state.tape = self
        try:
            yield
        finally:
            _state.tape = prev
            self.mode = prev_mode

    def recording(self):  # type: ignore[no-untyped-def]
        self.entries.clear()
        self.cursor = 0
        return self._activate('record')

    def replaying(self):  # type: ignore[no-untyped-def]
        self.cursor = 0
        return self._activate('replay')


def current_tape() -> Optional[RngTape]:
    return _state.tape


def reserve(device: torch.device, increment: int) -> SeedOffset:
    """Reserve ``increment`` Philox counters from ``device``'s generator: ``(seed, offset)``."""
    return _reserve(device, (int(increment) + 3) // 4 * 4)


def _reserve(device: torch.device, increment: int) -> SeedOffset:
    """Reserve ``increment`` Philox counters from the device generator."""
    if device.type == 'cuda':
        index = device.index if device.index is not None else torch.cuda.current_device()
        gen = torch.cuda.default_generators[index]
        with _gen_lock:
            seed = gen.initial_seed()
            offset = gen.get_offset()
            gen.set_offset(offset + increment)
        return int(seed) & 0xFFFFFFFFFFFFFFFF, int(offset)
    # CPU: derive a fresh 62-bit seed from the CPU generator (so that
    # torch.manual_seed controls it); the offset space starts at 0.
    seed = int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())
    return seed, 0


def philox_pair(device: torch.device, increment: int) -> SeedOffset:
    """``(seed, offset)`` for one RNG op that consumes ``increment`` counters.

    Inside a recording tape the pair is appended to the tape; inside a
    replaying tape the next recorded pair is returned instead of drawing.
    """
    # Round up to a multiple of 4: one Philox call yields 4 x 32-bit values.
    increment = (int(increment) + 3) // 4 * 4
    tape = _state.tape
    if device.type == 'cuda' and torch.cuda.is_current_stream_capturing():
        # The pair becomes a constant of the captured kernels: every replay of the graph
        # would draw the same mask (parallel/graph.py refuses such partitions up front).
        raise RuntimeError('a framework RNG op drew random numbers inside a hipGraph '
                           'capture; its replays would repeat the same mask every step')
    if tape is not None and tape.mode == 'replay':
        if tape.cursor >= len(tape.entries):
            raise RuntimeError('RNG tape exhausted: recomputation drew more random '
                               'numbers than the checkpointed forward pass')
        pair = tape.entries[tape.cursor]
        tape.cursor += 1
        return pair
    pair = _reserve(device, increment)
    if tape is not None and tape.mode == 'record':
        tape.entries.append(pair)
    return pair


class PhiloxSlot:
    """Device-resident Philox state of one captured cell.

    ``state`` is an int64 ``[2]`` GPU tensor ``(seed, base offset)`` that the host fills
    before each replay; ``delta`` counts the counters drawn so far in the current
    :func:`slot_scope` (the per-call offsets relative to the base).
    """

    __slots__ = ('state', 'delta')

    def __init__(self, state: torch.Tensor) -> None:
        if state.dtype != torch.int64 or state.numel() != 2 or not state.is_cuda:
            raise ValueError('a Philox slot is an int64 [2] GPU tensor')
        self.state = state
        self.delta = 0


@contextmanager
def slot_scope(slot: PhiloxSlot) -> Generator[None, None, None]:
    """RNG ops of this thread draw from ``slot`` (counters from 0) until the scope ends."""
    prev = _state.slot
    slot.delta = 0
    _state.slot = slot
    try:
        yield
    finally:
        _state.slot = prev


def philox_draw(device: torch.device,
                increment: int) -> Tuple[int, int, Optional[torch.Tensor]]:
    """``(seed, offset, rng)`` for one RNG op consuming ``increment`` counters.

    Inside a :func:`slot_scope` on a GPU: ``rng`` is the slot's device state and
    ``offset`` the op's position in the cell (``seed`` unused).  Otherwise ``rng`` is
    ``None`` and ``(seed, offset)`` is :func:`philox_pair`'s.
    """
    slot = _state.slot
    if slot is not None and device.type == 'cuda':
        delta = slot.delta
        slot.delta += (int(increment) + 3) // 4 * 4
        return 0, delta, slot.state
    seed, offset = philox_pair(device, increment)
    return seed, offset, None
