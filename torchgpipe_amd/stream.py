"""Device / stream abstraction (layer L1).

One API over HIP streams (``torch.cuda.Stream`` on ROCm *is* a HIP stream) and
a CPU sentinel so that the whole pipeline runtime can be exercised on CPU-only
machines by repeating ``'cpu'`` as a device.

Parity: ``torchgpipe/stream.py:12-101`` (CPUStream, new/current/default
stream, use_device/use_stream, wait_stream, record_stream).  Differences:

* ``wait_stream`` is ``torch.cuda.Stream.wait_stream`` (a HIP event record on the
  target + ``hipStreamWaitEvent`` on the source, asynchronous for the host); a CPU
  waiter synchronises on the target stream instead.
* A small per-device **stream pool** (``StreamPool``) replaces "``chunks``
  streams per device" (the reference allocates ``chunks`` copy streams per
  device, 1667 for ResNet p2).  Ordering is carried by events, so stream
  identity does not matter and a pool of a few streams per device suffices.
"""
from contextlib import contextmanager
import threading
from typing import Dict, Generator, List, Tuple, Union

import torch

__all__: List[str] = []


class _CPUStreamType:
    """Placeholder stream for the CPU device (no asynchronous queue)."""

    __slots__ = ()

    def __repr__(self) -> str:
        return '<CPUStream>'


CPUStream = _CPUStreamType()

AbstractStream = Union['torch.cuda.Stream', _CPUStreamType]


def _is_gpu_device(device: torch.device) -> bool:
    return device.type == 'cuda'


def is_cuda(stream: AbstractStream) -> bool:
    """True if ``stream`` is a real (HIP) device stream."""
    return stream is not CPUStream


def as_cuda(stream: AbstractStream) -> 'torch.cuda.Stream':
    return stream  # type: ignore[return-value]


def new_stream(device: torch.device) -> AbstractStream:
    if not _is_gpu_device(device):
        return CPUStream
    return torch.cuda.Stream(device)


def current_stream(device: torch.device) -> AbstractStream:
    if not _is_gpu_device(device):
        return CPUStream
    return torch.cuda.current_stream(device)


def default_stream(device: torch.device) -> AbstractStream:
    if not _is_gpu_device(device):
        return CPUStream
    return torch.cuda.default_stream(device)


@contextmanager
def use_device(device: torch.device) -> Generator[None, None, None]:
    if not _is_gpu_device(device):
        yield
        return
    with torch.cuda.device(device):
        yield


@contextmanager
def use_stream(stream: AbstractStream) -> Generator[None, None, None]:
    if not is_cuda(stream):
        yield
        return
    with torch.cuda.stream(as_cuda(stream)):
        yield


def get_device(stream: AbstractStream) -> torch.device:
    if is_cuda(stream):
        return as_cuda(stream).device
    return torch.device('cpu')


def wait_stream(source: AbstractStream, target: AbstractStream) -> None:
    """Make ``source`` wait until all work queued so far on ``target`` is done.

    * GPU waits GPU: event record on ``target`` + ``hipStreamWaitEvent`` on
      ``source`` (asynchronous for the host).
    * CPU waits GPU: host synchronises on ``target``.
    * anything waits CPU: nothing to do (CPU work is already complete).
    """
    if not is_cuda(target):
        return
    if is_cuda(source):
        as_cuda(source).wait_stream(as_cuda(target))
    else:
        as_cuda(target).synchronize()


def record_stream(tensor: torch.Tensor, stream: AbstractStream) -> None:
    """Tell the caching allocator that ``tensor`` is in use on ``stream``."""
    if is_cuda(stream) and tensor.is_cuda:
        tensor.record_stream(as_cuda(stream))


class StreamPool:
    """A fixed-size pool of side streams per device, handed out round-robin.

    Copy streams in the reference are indexed ``copy_streams[j][i]`` (one per
    micro-batch).  Here ``get(device, i)`` maps micro-batch ``i`` onto a
    small ring of streams; correctness only needs that the stream used to copy
    micro-batch ``i`` into partition ``j`` is the same one that its ``Wait``
    synchronises with, which the modulo mapping guarantees.

    Why a ring of 4 by default: a HIP process gets ``GPU_MAX_HW_QUEUES`` (4) hardware
    queues per device, so streams beyond that are multiplexed onto the same queues
    anyway, and in the fill-drain schedule at most ~2 micro-batches per device are in
    flight on the copy path at once.  Micro-batches ``i`` and ``i + 4`` then share a stream,
    which only adds ordering between copies that the clock schedule already orders.
    ``GPipe(copy_streams_per_device=chunks)`` restores the reference's one stream per
    micro-batch; ``tests/test_gpu_pipeline.py::test_copy_stream_ring_size_is_transparent``
    checks that rings of 1, 4 and ``chunks`` give identical training gradients.
    """

    def __init__(self, size: int = 4) -> None:
        self.size = max(1, int(size))
        self._streams: Dict[torch.device, List[AbstractStream]] = {}
        self._lock = threading.Lock()

    def get(self, device: torch.device, index: int) -> AbstractStream:
        if not _is_gpu_device(device):
            return CPUStream
        with self._lock:
            ring = self._streams.get(device)
            if ring is None:
                ring = [new_stream(device) for _ in range(self.size)]
                self._streams[device] = ring
        return ring[index % self.size]

    def grid(self, devices: List[torch.device], chunks: int) -> List[List[AbstractStream]]:
        """``grid[j][i]`` = stream for partition ``j`` and micro-batch ``i``."""
        return [[self.get(d, i) for i in range(chunks)] for d in devices]


_NAMED: Dict[Tuple[torch.device, str], torch.cuda.Stream] = {}
_NAMED_LOCK = threading.Lock()


def named_stream(device: torch.device, name: str) -> torch.cuda.Stream:
    """The process's stream ``name`` on ``device`` (created once, then reused).

    The engine's side streams -- a stage's forward / recompute lanes, relay routes,
    capture streams -- are named rather than created per stage object, so a process that
    builds many stages (``bench.py`` times several in a row) keeps a fixed set of streams,
    which is what the hardware-queue count of a multi-rank run is sized for
    (``parallel/stage.py`` ``stream_census``): ``torch.cuda.Stream()`` hands out a small
    pool round-robin, and ever new lanes would come to share pool streams, and with them
    hardware queues, with the RCCL communicators' streams.
    """
    key = (normalize_device(device), name)
    with _NAMED_LOCK:
        stream = _NAMED.get(key)
        if stream is None:
            stream = _NAMED[key] = torch.cuda.Stream(key[0])
    return stream


def normalize_device(device: torch.device) -> torch.device:
    """cuda → cuda:<current>, cpu:N → cpu.  Used to dedupe worker threads."""
    if device.type == 'cuda' and device.index is None:
        return torch.device('cuda', torch.cuda.current_device())
    if device.type == 'cpu' and device.index is not None:
        return torch.device('cpu')
    return device


def device_key(device: torch.device) -> Tuple[str, int]:
    d = normalize_device(device)
    return (d.type, -1 if d.index is None else d.index)
