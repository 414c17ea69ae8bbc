import pytest
import torch
from torch import nn

from torchgpipe_amd.skip import pop, skippable, stash
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker


@pytest.fixture(autouse=True)
def skip_tracker():
    tracker = SkipTracker()
    with use_skip_tracker(tracker):
        yield tracker


def test_stash(skip_tracker):
    @skippable(stash=['foo'])
    class Stash(nn.Module):
        def forward(self, x):
            yield stash('foo', x)
            return x * 2

    l1 = Stash()
    assert len(skip_tracker.tensors) == 0
    with use_skip_tracker(skip_tracker):
        l1(torch.tensor(42))
    assert len(skip_tracker.tensors) == 1


def test_pop():
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

    x = torch.tensor(42)
    out = Pop()(Stash()(x))
    assert out.item() == 42


def test_declare_but_not_use():
    @skippable(stash=['foo'])
    class Stash(nn.Module):
        def forward(self, x):
            return x * 2

    @skippable(pop=['foo'])
    class Pop(nn.Module):
        def forward(self, x):
            return x * 3

    with pytest.raises(RuntimeError, match="'foo' must be stashed but have not"):
        Stash()(torch.tensor(42))
    with pytest.raises(RuntimeError, match="'foo' has not been stashed"):
        Pop()(torch.tensor(42))


def test_pop_declared_but_not_popped(skip_tracker):
    @skippable(pop=['foo'])
    class Pop(nn.Module):
        def forward(self, x):
            return x * 3

    skip_tracker.save(None, None, 'foo', torch.tensor(1))
    with pytest.raises(RuntimeError, match="'foo' must be popped but have not"):
        Pop()(torch.tensor(42))


def test_stash_not_declared():
    @skippable()
    class Stash(nn.Module):
        def forward(self, x):
            yield stash('foo', x)
            return x * 2

    with pytest.raises(RuntimeError, match="'foo' has not been declared as stashable"):
        Stash()(torch.tensor(42))


def test_pop_not_declared():
    @skippable(stash=['foo'])
    class Stash(nn.Module):
        def forward(self, x):
            yield stash('foo', x)
            return x * 2

    @skippable()
    class Pop(nn.Module):
        def forward(self, x):
            foo = yield pop('foo')
            return foo

    latent = Stash()(torch.tensor(42))
    with pytest.raises(RuntimeError, match="'foo' has not been declared as poppable"):
        Pop()(latent)


def test_pop_not_stashed():
    @skippable(pop=['foo'])
    class Pop(nn.Module):
        def forward(self, x):
            yield pop('foo')

    with pytest.raises(RuntimeError):
        Pop()(torch.tensor(42))


def test_stash_none():
    @skippable(stash=['foo'])
    class Stash(nn.Module):
        def forward(self, x):
            yield stash('foo', None)
            return x * 2

    Stash()(torch.tensor(42))


def test_unknown_command():
    @skippable()
    class Bad(nn.Module):
        def forward(self, x):
            yield 'not a command'
            return x

    with pytest.raises(TypeError, match='is not a command from @skippable'):
        Bad()(torch.tensor(1))
