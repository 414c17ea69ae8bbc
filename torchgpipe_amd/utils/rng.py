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
"""
from contextlib import contextmanager
import threading
from typing import Generator, List, Optional, Tuple

import torch

__all__ = ['RngTape', 'philox_pair', 'current_tape']

SeedOffset = Tuple[int, int]


class _TapeState(threading.local):
    def __init__(self) -> None:
        self.tape: Optional['RngTape'] = None


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
