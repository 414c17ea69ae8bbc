"""Per-device worker threads (layer L4).

Parity: ``torchgpipe/worker.py:30-150`` (Task, worker loop, spawn_workers).

Difference by design: the reference spawns fresh threads on *every*
``GPipe.forward`` (``pipeline.py:112``).  Here a :class:`WorkerPool` keeps
one persistent daemon thread per distinct device for the lifetime of the
``GPipe`` module (``spawn_workers`` is kept as a context manager for
one-shot use and tests).  Each task carries its own grad mode so the
persistent threads honour ``torch.no_grad()`` of the calling thread.

Kernel launches are asynchronous, so a worker thread only spends host time
enqueueing HIP work; the device threads let PyTorch issue launches for
different GPUs concurrently (PyTorch releases the GIL inside its C++ ops).
"""
import atexit
from contextlib import contextmanager
from queue import Queue
import sys
from threading import Thread
from types import TracebackType
from typing import Callable, Dict, Generator, List, Optional, Tuple, Type, Union
import weakref

import torch

from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.stream import AbstractStream, normalize_device, use_device, use_stream

__all__: List[str] = []

ExcInfo = Tuple[Type[BaseException], BaseException, TracebackType]
InQueue = Queue
OutQueue = Queue


class Task:
    """``compute`` runs on a worker thread; ``finalize`` on the scheduling thread."""

    __slots__ = ('stream', '_compute', '_finalize', 'grad_mode')

    def __init__(self, stream: AbstractStream, *,
                 compute: Callable[[], Batch],
                 finalize: Optional[Callable[[Batch], None]]) -> None:
        self.stream = stream
        self._compute = compute
        self._finalize = finalize
        self.grad_mode = torch.is_grad_enabled()

    def compute(self) -> Batch:
        with use_stream(self.stream):
            return self._compute()

    def finalize(self, batch: Batch) -> None:
        if self._finalize is None:
            return
        with use_stream(self.stream):
            self._finalize(batch)


def worker(in_queue: InQueue, out_queue: OutQueue, device: torch.device,
           grad_mode: Optional[bool] = None) -> None:
    """Main loop of a device thread.  ``None`` in the queue terminates it."""
    if grad_mode is not None:
        torch.set_grad_enabled(grad_mode)
    with use_device(device):
        while True:
            task = in_queue.get()
            if task is None:
                break
            try:
                with torch.set_grad_enabled(task.grad_mode if grad_mode is None else grad_mode):
                    batch = task.compute()
            except Exception:
                out_queue.put((False, sys.exc_info()))
                task = None
                continue
            out_queue.put((True, (task, batch)))
            # a parked persistent thread must not keep the last task (its closure holds the
            # partition, and through it the module and its caches) alive until the next one
            task = batch = None
    out_queue.put((False, None))


def _start(device: torch.device, grad_mode: Optional[bool]) -> Tuple[InQueue, OutQueue, Thread]:
    in_queue: InQueue = Queue()
    out_queue: OutQueue = Queue()
    t = Thread(target=worker, args=(in_queue, out_queue, device, grad_mode), daemon=True,
               name=f'gpipe-worker-{device}')
    t.start()
    return in_queue, out_queue, t


def _drain_close(queues: Dict[torch.device, Tuple[InQueue, OutQueue]]) -> None:
    for in_q, _ in queues.values():
        in_q.put(None)
    running = {id(out_q): out_q for _, out_q in queues.values()}
    while running:
        key, out_q = running.popitem()
        ok, payload = out_q.get()
        if not ok and payload is None:
            continue
        running[key] = out_q


_live_pools: 'weakref.WeakSet[WorkerPool]' = weakref.WeakSet()


@atexit.register
def _close_live_pools() -> None:
    # Join idle device threads before interpreter finalisation: a daemon thread
    # that still owns a HIP context while C++ static destructors run aborts the
    # process ("terminate called without an active exception").
    for pool in list(_live_pools):
        try:
            pool.close(wait=True)
        except Exception:  # pragma: no cover
            pass


class WorkerPool:
    """Persistent device threads shared by every forward of one ``GPipe``."""

    def __init__(self) -> None:
        self._workers: Dict[torch.device, Tuple[InQueue, OutQueue]] = {}
        self._threads: List[Thread] = []
        _live_pools.add(self)

    def queues(self, devices: List[torch.device]) -> Tuple[List[InQueue], List[OutQueue]]:
        in_queues: List[InQueue] = []
        out_queues: List[OutQueue] = []
        for device in devices:
            device = normalize_device(device)
            pair = self._workers.get(device)
            if pair is None:
                in_q, out_q, t = _start(device, None)
                pair = (in_q, out_q)
                self._workers[device] = pair
                self._threads.append(t)
            in_queues.append(pair[0])
            out_queues.append(pair[1])
        return in_queues, out_queues

    def close(self, wait: bool = True) -> None:
        """Stop the threads; ``wait`` joins them (never from a finalizer)."""
        if self._workers:
            if wait:
                _drain_close(self._workers)
                for t in self._threads:
                    t.join(timeout=10)
            else:
                for in_q, _ in self._workers.values():
                    in_q.put(None)
            self._workers = {}
            self._threads = []

    def __del__(self) -> None:  # pragma: no cover - interpreter shutdown order
        try:
            self.close(wait=False)
        except Exception:
            pass


@contextmanager
def spawn_workers(devices: List[torch.device],
                  ) -> Generator[Tuple[List[InQueue], List[OutQueue]], None, None]:
    """Spawn one thread per distinct device for the duration of the context."""
    workers: Dict[torch.device, Tuple[InQueue, OutQueue]] = {}
    in_queues: List[InQueue] = []
    out_queues: List[OutQueue] = []
    grad_mode = torch.is_grad_enabled()
    for device in devices:
        device = normalize_device(device)
        pair = workers.get(device)
        if pair is None:
            in_q, out_q, _ = _start(device, grad_mode)
            pair = (in_q, out_q)
            workers[device] = pair
        in_queues.append(pair[0])
        out_queues.append(pair[1])
    try:
        yield in_queues, out_queues
    finally:
        _drain_close(workers)


Payload = Union[Tuple[Task, Batch], ExcInfo, None]
