"""GPipe fill-drain scheduler for one process driving several devices (layer L4).

Parity: ``torchgpipe/pipeline.py:36-249``.

Forward runs the anti-diagonal clock-cycle schedule: at clock ``k`` every
cell ``(i, j)`` with ``i + j == k`` (micro-batch ``i`` on partition ``j``)
runs concurrently on its device thread.  Each clock cycle ends with a host
barrier (lock-step), but that barrier only covers kernel *launch*; device
work is ordered by stream events, so GPUs run ahead of the host.

There is no backward scheduler: ``fence`` and ``compute`` build an autograd
graph whose edges encode the schedule, and PyTorch's autograd engine (one
thread per device) executes it.  Per cell the graph is::

    Copy → Wait(copy→compute) → Checkpoint → Wait(compute→copy)
         → Fork → Recompute → Join → Copy(next partition) ...

plus ``depend`` edges (Fork on micro-batch ``i-1`` → Join on ``i``) so that on
each partition micro-batch ``i-1`` back-propagates after micro-batch ``i``,
and ``Recompute`` sits in front of the gradient ``Wait`` so recomputation
overlaps the incoming gradient transfer.
"""
from typing import Callable, Iterable, List, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor, nn

from torchgpipe_amd.checkpoint import Checkpointing
from torchgpipe_amd.copy import Copy, Wait
from torchgpipe_amd.dependency import fork, join
from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.skip.layout import SkipLayout, inspect_skip_layout
from torchgpipe_amd.skip.tracker import SkipTrackerThroughPotals, use_skip_tracker
from torchgpipe_amd.stream import AbstractStream, current_stream, use_device
from torchgpipe_amd.utils import trace
from torchgpipe_amd.worker import InQueue, OutQueue, Task, spawn_workers

__all__: List[str] = []

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]


def depend(fork_from: Batch, join_to: Batch) -> None:
    """Backward of ``join_to`` must finish before backward of ``fork_from``."""
    fork_from[0], phony = fork(fork_from[0])
    join_to[0] = join(join_to[0], phony)


def copy(batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream) -> None:
    batch[:] = Copy.apply(prev_stream, next_stream, *batch)


def wait(batch: Batch, prev_stream: AbstractStream, next_stream: AbstractStream) -> None:
    batch[:] = Wait.apply(prev_stream, next_stream, *batch)


def clock_cycles(m: int, n: int) -> Iterable[List[Tuple[int, int]]]:
    """Yield the cells ``(i, j)`` of each clock cycle of an ``m × n`` pipeline.

    ::

        k  cells
        0  (0,0)
        1  (1,0) (0,1)
        2  (2,0) (1,1) (0,2)
        3        (2,1) (1,2)
        4              (2,2)
    """
    for k in range(m + n - 1):
        lo = max(0, k - m + 1)
        hi = min(k, n - 1)
        yield [(k - j, j) for j in range(lo, hi + 1)]


class Pipeline:
    """Runs ``partitions`` over ``batches`` in place (single process)."""

    def __init__(self,
                 batches: List[Batch],
                 partitions: List[nn.Sequential],
                 devices: Optional[List[torch.device]] = None,
                 copy_streams: Optional[List[List[AbstractStream]]] = None,
                 skip_layout: Optional[SkipLayout] = None,
                 checkpoint_stop: int = 0,
                 queues: Optional[Tuple[List[InQueue], List[OutQueue]]] = None,
                 on_output: Optional[Callable[[int, Batch, AbstractStream], None]] = None,
                 lanes: Optional[Sequence[Optional[Sequence[AbstractStream]]]] = None,
                 ) -> None:
        self.batches = batches
        self.partitions = partitions
        if devices is None:
            devices = [torch.device('cpu') for _ in partitions]
        self.devices = devices
        if copy_streams is None:
            copy_streams = [[current_stream(d)] * len(batches) for d in devices]
        self.copy_streams = copy_streams
        if skip_layout is None:
            skip_layout = inspect_skip_layout(partitions)
        self.skip_layout = skip_layout
        self.checkpoint_stop = checkpoint_stop
        self._queues = queues
        # called with (i, batch, stream that computed it) as micro-batch i leaves the last
        # partition (K11 gather)
        self.on_output = on_output
        # forward lanes per partition (GPipe(overlap_forward=True)): cell (i, j) computes on
        # lanes[j][i % 2] instead of device j's current stream, so consecutive micro-batches
        # of a stateless partition overlap on the GPU wherever their inputs are ready
        self.lanes = lanes

    def run(self) -> None:
        m = len(self.batches)
        n = len(self.partitions)
        trackers = [SkipTrackerThroughPotals(self.skip_layout) for _ in range(m)]

        if self._queues is not None:
            in_queues, out_queues = self._queues
            for schedule in clock_cycles(m, n):
                self.fence(schedule, trackers)
                self.compute(schedule, trackers, in_queues, out_queues)
            return

        with spawn_workers(self.devices) as (in_queues, out_queues):
            for schedule in clock_cycles(m, n):
                self.fence(schedule, trackers)
                self.compute(schedule, trackers, in_queues, out_queues)

    def fence(self, schedule: List[Tuple[int, int]],
              skip_trackers: List[SkipTrackerThroughPotals]) -> None:
        """Wire dependencies and copies for this cycle (scheduling thread)."""
        batches = self.batches
        copy_streams = self.copy_streams
        for i, j in schedule:
            if i != 0:
                depend(batches[i - 1], batches[i])
            next_stream = copy_streams[j][i]
            # every skip from one source partition into j travels as one packed hop
            for prev_j, keys in self.skip_layout.copy_groups(j):
                skip_trackers[i].copy_many(batches[i], copy_streams[prev_j][i], next_stream,
                                           keys)
            if j != 0:
                copy(batches[i], copy_streams[j - 1][i], next_stream)

    def compute(self, schedule: List[Tuple[int, int]],
                skip_trackers: List[SkipTrackerThroughPotals],
                in_queues: List[InQueue], out_queues: List[OutQueue]) -> None:
        batches = self.batches
        partitions = self.partitions
        devices = self.devices
        copy_streams = self.copy_streams
        n = len(partitions)
        streams = [current_stream(d) for d in devices]

        run = {}
        for i, j in schedule:
            batch = batches[i]
            lane = self.lanes[j] if self.lanes is not None else None
            stream = run[(i, j)] = lane[i % 2] if lane else streams[j]
            if j != 0:
                wait(batch, copy_streams[j][i], stream)
            elif lane:
                # the mini-batch was made on the device's current stream (and its gradient
                # goes back there)
                wait(batch, streams[j], stream)
            task = self._make_task(i, j, batch, partitions[j], skip_trackers[i], stream)
            in_queues[j].put(task)

        exc_info = None
        for i, j in schedule:
            ok, payload = out_queues[j].get()
            if exc_info is not None:
                continue
            if not ok:
                exc_info = payload
                continue
            task, batch = payload
            if j != n - 1:
                wait(batch, run[(i, j)], copy_streams[j][i])
            with use_device(devices[j]):
                task.finalize(batch)
                if j == n - 1 and self.on_output is not None:
                    self.on_output(i, batch, run[(i, j)])
            batches[i] = batch

        if exc_info is not None:
            raise exc_info[1].with_traceback(exc_info[2])

    def _make_task(self, i: int, j: int, batch: Batch, partition: nn.Sequential,
                   tracker: SkipTrackerThroughPotals, stream: AbstractStream) -> Task:
        label = f'fwd mb{i} p{j}'

        def run(input: TensorOrTensors) -> TensorOrTensors:
            with use_skip_tracker(tracker), trace.range(label):
                return partition(input)

        if i < self.checkpoint_stop:
            chk = Checkpointing(run, batch)
            return Task(stream, compute=chk.checkpoint, finalize=chk.recompute)

        compute: Callable[[], Batch] = lambda: batch.call(run)  # noqa: E731
        return Task(stream, compute=compute, finalize=None)
