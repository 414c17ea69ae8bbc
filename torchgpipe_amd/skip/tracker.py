"""Per-thread trackers of stashed skip tensors.

Parity: ``torchgpipe/skip/tracker.py:19-179``.

* :class:`SkipTracker` — a plain dict; used when a skippable module runs
  outside ``GPipe`` (e.g. in a plain ``nn.Sequential`` or under
  ``nn.DataParallel``).
* :class:`SkipTrackerThroughPotals` — one per micro-batch inside ``GPipe``:
  skips that stay within a partition use the dict; skips that cross
  partitions are hidden in :class:`~torchgpipe_amd.skip.portal.Portal`s and
  tied to the micro-batch lane with Fork/Join so backward stays ordered.
  (The class name keeps the reference's spelling for API compatibility;
  ``SkipTrackerThroughPortals`` is provided as an alias.)
"""
from contextlib import contextmanager
import threading
from typing import Dict, Generator, List, Optional, Sequence, Tuple

from torch import Tensor

from torchgpipe_amd.checkpoint import is_checkpointing
from torchgpipe_amd.dependency import fork, join
from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.skip.layout import SkipLayout
from torchgpipe_amd.skip.namespace import Namespace
from torchgpipe_amd.skip.portal import Portal, copy_portals
from torchgpipe_amd.stream import AbstractStream

__all__: List[str] = []

Key = Tuple[Namespace, str]


class SkipTracker:
    def __init__(self) -> None:
        self.tensors: Dict[Key, Optional[Tensor]] = {}

    def save(self, batch: Batch, ns: Namespace, name: str, tensor: Optional[Tensor]) -> None:
        self.tensors[(ns, name)] = tensor

    def load(self, batch: Batch, ns: Namespace, name: str) -> Optional[Tensor]:
        return self.tensors.pop((ns, name))

    def copy(self, batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream,
             ns: Namespace, name: str) -> None:
        raise TypeError('copy is not supported for non-portal skip tensors')

    def copy_many(self, batch: Batch, prev_stream: AbstractStream,
                  next_stream: AbstractStream, keys: Sequence[Key]) -> None:
        raise TypeError('copy is not supported for non-portal skip tensors')


class SkipTrackerThroughPotals(SkipTracker):
    def __init__(self, skip_layout: SkipLayout) -> None:
        super().__init__()
        self.skip_layout = skip_layout
        self.portals: Dict[Key, Portal] = {}

    def save(self, batch: Batch, ns: Namespace, name: str, tensor: Optional[Tensor]) -> None:
        if not self.skip_layout.requires_copy(ns, name):
            super().save(batch, ns, name, tensor)
            return
        key = (ns, name)
        portal = self.portals.get(key)
        if portal is None:
            # life 3 under checkpointing (freed by the recomputed PortalOrange),
            # life 2 otherwise (freed by the first PortalOrange).
            portal = Portal(tensor, 3 if is_checkpointing() else 2)
            self.portals[key] = portal
        else:
            # Recomputation re-stashes into the existing portal; free it at the
            # recomputed blue().
            portal.put_tensor(tensor, 1)
        phony = portal.blue()
        batch[0] = join(batch[0], phony)

    def load(self, batch: Batch, ns: Namespace, name: str) -> Optional[Tensor]:
        if not self.skip_layout.requires_copy(ns, name):
            return super().load(batch, ns, name)
        portal = self.portals[(ns, name)]
        batch[0], phony = fork(batch[0])
        return portal.orange(phony)

    def copy(self, batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream,
             ns: Namespace, name: str) -> None:
        self.copy_many(batch, prev_stream, next_stream, [(ns, name)])

    def copy_many(self, batch: Batch, prev_stream: AbstractStream,
                  next_stream: AbstractStream, keys: Sequence[Key]) -> None:
        """Move the portals of ``keys`` (one source partition, one destination) as one
        hop, packed into a single transfer between two GPUs."""
        assert all(self.skip_layout.requires_copy(ns, name) for ns, name in keys)
        batch[0], phony = fork(batch[0])
        phony = copy_portals([self.portals[key] for key in keys], prev_stream, next_stream,
                             phony)
        batch[0] = join(batch[0], phony)


SkipTrackerThroughPortals = SkipTrackerThroughPotals


class _Local(threading.local):
    def __init__(self) -> None:
        self.skip_tracker: Optional[SkipTracker] = None


_local = _Local()


@contextmanager
def use_skip_tracker(skip_tracker: SkipTracker) -> Generator[None, None, None]:
    prev = _local.skip_tracker
    _local.skip_tracker = skip_tracker
    try:
        yield
    finally:
        _local.skip_tracker = prev


def current_skip_tracker() -> SkipTracker:
    tracker = _local.skip_tracker
    if tracker is None:
        tracker = SkipTracker()
        _local.skip_tracker = tracker
    return tracker
