from queue import Queue
import threading

import torch
from torch import nn

from torchgpipe_amd.checkpoint import enable_checkpointing, enable_recomputing
from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.skip import pop, skippable, stash
from torchgpipe_amd.skip.layout import SkipLayout
from torchgpipe_amd.skip.tracker import (SkipTracker, SkipTrackerThroughPortals,
                                         SkipTrackerThroughPotals, current_skip_tracker,
                                         use_skip_tracker)


def test_default_skip_tracker_is_plain_and_per_thread():
    q = Queue()
    t = threading.Thread(target=lambda: q.put(current_skip_tracker()))
    t.start()
    t.join()
    tracker = q.get()
    assert type(tracker) is SkipTracker
    assert tracker is not current_skip_tracker()


def test_alias():
    assert SkipTrackerThroughPortals is SkipTrackerThroughPotals


def test_skippable_in_plain_sequential_uses_default_tracker():
    @skippable(stash=['foo'])
    class Stash(nn.Module):
        def forward(self, x):
            yield stash('foo', x)
            return x * 2

    @skippable(pop=['foo'])
    class Pop(nn.Module):
        def forward(self, x):
            foo = yield pop('foo')
            return foo

    x = torch.rand(10)
    assert torch.allclose(nn.Sequential(Stash(), Pop())(x), x)


def test_reuse_portal():
    layout = SkipLayout(num_partitions=2, skip_routes={(None, 'test'): (0, 1)})
    tracker = SkipTrackerThroughPotals(layout)
    batch = Batch(torch.tensor([1.0]))
    tracker.save(batch, None, 'test', torch.tensor([2.0]))
    portal = tracker.portals[(None, 'test')]
    tracker.save(batch, None, 'test', torch.tensor([2.0]))
    assert portal is tracker.portals[(None, 'test')]


def test_no_copy_no_portal():
    layout = SkipLayout(num_partitions=2, skip_routes={(None, 'copy'): (0, 1),
                                                       (None, 'not_copy'): (0, 0)})
    tracker = SkipTrackerThroughPotals(layout)
    batch = Batch(torch.tensor([1.0]))
    tracker.save(batch, None, 'copy', torch.tensor([2.0]))
    tracker.save(batch, None, 'not_copy', torch.tensor([2.0]))
    assert (None, 'copy') in tracker.portals and (None, 'copy') not in tracker.tensors
    assert (None, 'not_copy') in tracker.tensors and (None, 'not_copy') not in tracker.portals


def test_tensor_life_without_checkpointing():
    layout = SkipLayout(num_partitions=2, skip_routes={(None, 'test'): (0, 1)})
    tracker = SkipTrackerThroughPotals(layout)
    batch = Batch(torch.tensor([1.0]))
    tracker.save(batch, None, 'test', torch.tensor([2.0]))
    assert tracker.portals[(None, 'test')].tensor_life == 1
    tracker.load(batch, None, 'test')
    assert tracker.portals[(None, 'test')].tensor_life == 0


def test_tensor_life_with_checkpointing():
    layout = SkipLayout(num_partitions=2, skip_routes={(None, 'test'): (0, 1)})
    tracker = SkipTrackerThroughPotals(layout)
    batch = Batch(torch.tensor([1.0]))
    t = torch.tensor([2.0])
    with enable_checkpointing():
        tracker.save(batch, None, 'test', t)
    assert tracker.portals[(None, 'test')].tensor_life == 2
    with enable_checkpointing():
        tracker.load(batch, None, 'test')
    assert tracker.portals[(None, 'test')].tensor_life == 1
    with enable_recomputing():
        tracker.load(batch, None, 'test')
    assert tracker.portals[(None, 'test')].tensor_life == 0
    with enable_recomputing():
        tracker.save(batch, None, 'test', t)
    assert tracker.portals[(None, 'test')].tensor_life == 0


def test_copy_is_not_supported_for_plain_tracker():
    import pytest
    with pytest.raises(TypeError, match='copy is not supported for non-portal skip tensors'):
        SkipTracker().copy(Batch(torch.rand(1)), None, None, None, 'x')


def test_use_skip_tracker_restores_previous():
    outer = current_skip_tracker()
    inner = SkipTracker()
    with use_skip_tracker(inner):
        assert current_skip_tracker() is inner
    assert current_skip_tracker() is outer
