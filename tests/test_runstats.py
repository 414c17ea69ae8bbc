"""OrderedRunningStats (torchgpipe_amd/runstats.py): slotted BatchNorm updates folded in
issue order give the running statistics of the plain sequential updates."""
import copy

import pytest
import torch
from torch import nn

from torchgpipe_amd.batchnorm import DeferredBatchNorm
from torchgpipe_amd.runstats import OrderedRunningStats


class _Net(nn.Module):
    def __init__(self) -> None:
        super().__init__()
        self.conv = nn.Conv2d(3, 6, 3, padding=1)
        self.bn1 = nn.BatchNorm2d(6, momentum=0.1)
        self.bn2 = nn.BatchNorm2d(6, momentum=0.3)
        self.bn3 = nn.BatchNorm1d(5)

    def forward(self, x: torch.Tensor, skip_bn2: bool = False) -> torch.Tensor:
        y = self.bn1(self.conv(x))
        if not skip_bn2:
            y = self.bn2(y)
        return self.bn3(y.mean((2, 3))[:, :5])


def _buffers(m: nn.Module):
    return {k: v.clone() for k, v in m.named_buffers()}


@pytest.mark.parametrize('updates', [1, 5, 37])
def test_fold_matches_sequential_updates(updates):
    torch.manual_seed(0)
    a = _Net()
    with torch.no_grad():  # non-trivial starting statistics
        for bn in (a.bn1, a.bn2, a.bn3):
            bn.running_mean.uniform_(-1, 1)
            bn.running_var.uniform_(0.5, 2)
    b = copy.deepcopy(a)
    xs = [torch.randn(4, 3, 8, 8) * (1 + k) + k for k in range(updates)]
    skips = [k % 3 == 1 for k in range(updates)]  # bn2 misses some updates
    for x, skip in zip(xs, skips):
        a(x, skip)
    slots = OrderedRunningStats.for_module(b)
    assert slots is not None
    slots.begin(updates + 2)
    for x, skip in zip(xs, skips):
        with slots.update():
            b(x, skip)
    slots.commit()
    want, got = _buffers(a), _buffers(b)
    for k in want:
        if k.endswith('num_batches_tracked'):
            assert torch.equal(got[k], want[k]), k
        else:
            torch.testing.assert_close(got[k], want[k], rtol=1e-5, atol=1e-6, msg=k)
    # the real buffers (same tensor objects) are back in place, momentum restored
    assert b.bn2.momentum == 0.3 and b.bn1.momentum == 0.1
    assert b.bn1.running_mean.data_ptr() == dict(b.named_buffers())['bn1.running_mean'].data_ptr()


def test_buffers_are_swapped_only_inside_an_update():
    net = _Net()
    ids = {k: v.data_ptr() for k, v in net.named_buffers()}
    slots = OrderedRunningStats.for_module(net)
    slots.begin(2)
    with slots.update():
        assert net.bn1.running_mean.data_ptr() != ids['bn1.running_mean']
        assert net.bn1.momentum == 1.0
    assert {k: v.data_ptr() for k, v in net.named_buffers()} == ids
    with pytest.raises(RuntimeError):
        with slots.update():
            pass
        with slots.update():
            pass
        with slots.update():  # a third update: only two slots
            pass
    slots.commit()


def test_eval_mode_batchnorms_are_left_alone():
    torch.manual_seed(1)
    a = _Net()
    a.bn2.eval()
    b = copy.deepcopy(a)
    x = torch.randn(4, 3, 8, 8)
    a(x)
    slots = OrderedRunningStats.for_module(b)
    slots.begin(1)
    with slots.update():
        out = b(x)
    slots.commit()
    assert torch.isfinite(out).all()
    for k, v in _buffers(a).items():  # bn2 untouched, bn1 / bn3 folded
        torch.testing.assert_close(dict(b.named_buffers())[k], v, rtol=1e-5, atol=1e-6, msg=k)
    all_eval = copy.deepcopy(b).eval()
    s2 = OrderedRunningStats.for_module(all_eval)
    s2.begin(1)
    assert not s2.active


def test_ineligible_modules():
    assert OrderedRunningStats.for_module(nn.Linear(2, 2)) is None
    assert OrderedRunningStats.for_module(nn.BatchNorm2d(3, momentum=None)) is None
    assert OrderedRunningStats.for_module(DeferredBatchNorm(3)) is None
    assert OrderedRunningStats.for_module(nn.BatchNorm2d(3, track_running_stats=False)) is None
