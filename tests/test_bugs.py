import pytest
import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd import GPipe


def test_python_autograd_function():
    # Identity autograd functions must detach before returning, otherwise
    # autograd refuses views sharing storage with grad-requiring inputs.
    class Identity(torch.autograd.Function):
        @staticmethod
        def forward(ctx, input):
            return input

        @staticmethod
        def backward(ctx, grad):
            return grad

    class M(nn.Module):
        def forward(self, x):
            return Identity.apply(x)

    model = GPipe(nn.Sequential(M(), M()), [1, 1], devices=['cpu', 'cpu'], checkpoint='always')
    x = torch.rand(42)
    assert torch.allclose(x, model(x))


def test_exception_no_hang():
    class Boom(Exception):
        pass

    class Pass(nn.Module):
        def forward(self, x):
            return x

    class Raise(nn.Module):
        def forward(self, x):
            raise Boom()

    model = GPipe(nn.Sequential(Pass(), Pass(), Raise()), [1, 1, 1], devices=['cpu'] * 3,
                  chunks=3)
    with pytest.raises(Boom):
        model(torch.rand(3))
    # ... and the persistent workers still serve the next call.
    with pytest.raises(Boom):
        model(torch.rand(3))


def test_parallel_randoms():
    class Dropouts(nn.Module):
        def forward(self, x):
            for _ in range(100):
                x = F.dropout(x, p=0.001)
            return x

    x = torch.rand(10, 10, requires_grad=True)
    model = GPipe(nn.Sequential(Dropouts(), Dropouts()), [1, 1], devices=['cpu', 'cpu'],
                  chunks=10, checkpoint='always')
    y = model(x)
    y.norm().backward()
    # Recomputation replays the same dropout masks: zero outputs <=> zero grads.
    assert y.to(torch.bool).tolist() == x.grad.to(torch.bool).tolist()
