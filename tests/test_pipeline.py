import time

import torch
from torch import nn

from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.pipeline import Pipeline, clock_cycles


def test_clock_cycles():
    assert list(clock_cycles(1, 1)) == [[(0, 0)]]
    assert list(clock_cycles(1, 3)) == [[(0, 0)], [(0, 1)], [(0, 2)]]
    assert list(clock_cycles(3, 1)) == [[(0, 0)], [(1, 0)], [(2, 0)]]
    assert list(clock_cycles(3, 3)) == [[(0, 0)], [(1, 0), (0, 1)], [(2, 0), (1, 1), (0, 2)],
                                        [(2, 1), (1, 2)], [(2, 2)]]
    assert list(clock_cycles(4, 2)) == [[(0, 0)], [(1, 0), (0, 1)], [(2, 0), (1, 1)],
                                        [(3, 0), (2, 1)], [(3, 1)]]


def test_clock_cycles_cover_every_cell_once():
    for m in range(1, 6):
        for n in range(1, 6):
            cells = [c for cycle in clock_cycles(m, n) for c in cycle]
            assert sorted(cells) == [(i, j) for i in range(m) for j in range(n)]
            for k, cycle in enumerate(clock_cycles(m, n)):
                assert all(i + j == k for i, j in cycle)


def test_forward_lockstep():
    timeline = []

    class DelayedLog(nn.Module):
        def __init__(self, j, seconds):
            super().__init__()
            self.i = 0
            self.j = j
            self.seconds = seconds

        def forward(self, x):
            time.sleep(self.seconds)
            timeline.append((self.i, self.j))
            self.i += 1
            return x

    batches = [Batch(torch.rand(1, 1)) for _ in range(3)]
    partitions = [nn.Sequential(DelayedLog(0, seconds=0)),
                  nn.Sequential(DelayedLog(1, seconds=0.1))]
    Pipeline(batches, partitions).run()
    # partition 0: 0! 1!    2!
    # partition 1:    000!  111! 222!
    assert timeline == [(0, 0), (1, 0), (0, 1), (2, 0), (1, 1), (2, 1)]
