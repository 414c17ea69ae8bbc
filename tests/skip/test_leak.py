import pytest
import torch
from torch import nn

from torchgpipe_amd import GPipe, is_checkpointing, is_recomputing
from torchgpipe_amd.skip import pop, skippable, stash
from torchgpipe_amd.skip.tracker import current_skip_tracker


@skippable(stash=['skip'])
class Stash(nn.Module):
    def forward(self, x):
        yield stash('skip', x)
        return x


@skippable(pop=['skip'])
class Pop(nn.Module):
    def forward(self, x):
        skip = yield pop('skip')
        return x + skip


def portal_life_is(life, tracker=None):
    tracker = tracker or current_skip_tracker()
    portal = list(tracker.portals.values())[0]
    if life == 0:
        return portal.tensor_life == 0 and portal.tensor is None
    return portal.tensor_life == life and portal.tensor is not None


@pytest.mark.parametrize('train', [True, False], ids=['train', 'eval'])
@pytest.mark.parametrize('checkpoint', ['always', 'except_last', 'never'])
def test_delete_portal_tensor(train, checkpoint):
    # without checkpointing: Stash(2→blue→1) Pop(1→orange→0)
    # with checkpointing:    Stash(3→2) Pop(2→1) Pop'(1→0) Stash'(1→0)
    stash_ = Stash()

    @stash_.register_forward_hook
    def after_stash(*_):
        if is_checkpointing():
            assert portal_life_is(2)
        elif is_recomputing():
            assert portal_life_is(0)
        else:
            assert portal_life_is(1)

    pop_ = Pop()

    @pop_.register_forward_hook
    def after_pop(*_):
        if is_checkpointing():
            assert portal_life_is(1)
        else:
            assert portal_life_is(0)

    class NoPortalTensorAtBackward(nn.Module):
        class F(torch.autograd.Function):
            @staticmethod
            def forward(ctx, x):
                ctx.tracker = current_skip_tracker()
                return x.detach()

            @staticmethod
            def backward(ctx, grad):
                assert portal_life_is(0, ctx.tracker)
                return grad

        def forward(self, x):
            return self.F.apply(x)

    model = GPipe(nn.Sequential(NoPortalTensorAtBackward(), stash_, pop_), balance=[2, 1],
                  devices=['cpu', 'cpu'], chunks=2, checkpoint=checkpoint)
    x = torch.rand(10, requires_grad=True)
    if train:
        model.train()
        model(x).norm().backward()
    else:
        model.eval()
        with torch.no_grad():
            model(x)


@pytest.mark.parametrize('train', [True, False], ids=['train', 'eval'])
def test_no_portal_without_gpipe(train, monkeypatch):
    def deny(*args, **kwargs):
        raise AssertionError('tried to create Portal without GPipe')

    monkeypatch.setattr('torchgpipe_amd.skip.portal.Portal.__init__', deny)
    model = nn.Sequential(Stash(), Pop())
    x = torch.rand(10, requires_grad=True)
    if train:
        model.train()
        model(x).norm().backward()
    else:
        model.eval()
        with torch.no_grad():
            model(x)
