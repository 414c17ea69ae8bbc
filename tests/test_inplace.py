import pytest
import torch
from torch import nn

from torchgpipe_amd import GPipe

LEAF_INPLACE = ('a leaf Variable that requires grad (is being|has been) used in an in-place '
                'operation.')


def test_inplace_on_requires_grad():
    model = GPipe(nn.Sequential(nn.Linear(1, 1), nn.ReLU(inplace=True)), [1, 1],
                  devices=['cpu', 'cpu'], checkpoint='always')
    y = model(torch.rand(1))
    with pytest.raises(RuntimeError, match=LEAF_INPLACE):
        y.backward()


@pytest.mark.xfail(strict=True)
def test_inplace_on_not_requires_grad():
    # An in-place op on a tensor that does not require grad cannot be detected
    # (documented limitation, same as the reference).
    model = GPipe(nn.Sequential(nn.ReLU(inplace=True)), [1], devices=['cpu'],
                  checkpoint='always')
    y = model(torch.rand(1))
    with pytest.raises(RuntimeError, match=LEAF_INPLACE):
        y.backward()


@pytest.mark.xfail(strict=True)
def test_inplace_incorrect_grad():
    class M(nn.Module):
        def forward(self, foo_bar):
            foo, bar = foo_bar
            bar.add_(1)  # not idempotent: recomputation applies it twice
            return foo * bar

    model = GPipe(nn.Sequential(M()), [1], devices=['cpu'], checkpoint='always')
    foo = torch.tensor([1.], requires_grad=True)
    bar = torch.tensor([1.])
    model((foo, bar)).backward()
    # The reference semantics would give 2; recomputation makes it 3.
    assert foo.grad.item() == 2
