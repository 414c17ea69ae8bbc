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


@pytest.mark.gpu
def test_every_tensor_of_a_tuple_is_fenced(gpu_sleep):
    """Wait must cover every tensor of a micro-batch, not only the first:
    a slow gradient on the second tensor has to be ordered before the copy
    stream sends it back."""
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')

    class SlowGrad(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x.detach()

        @staticmethod
        def backward(ctx, grad):
            with torch.cuda.device(grad.device):
                gpu_sleep(0.05)
            return grad

    class Fan(nn.Module):
        def forward(self, pair):
            a, b = pair
            return a * 1, b * 2, b * 3

    class Sum(nn.Module):
        def forward(self, triple):
            a, b, c = triple
            return a + SlowGrad.apply(b) + c

    devices = [0, 1] if torch.cuda.device_count() > 1 else [0, 0]
    model = GPipe(nn.Sequential(Fan(), Sum()), [1, 1], devices=devices, chunks=32,
                  checkpoint='never')
    a = torch.rand(1024, 3, 32, 32, device=0, requires_grad=True)
    b = torch.rand(1024, 3, 32, 32, device=0, requires_grad=True)
    model((a, b)).norm().backward()
    torch.cuda.synchronize()
    # d/db of |a + 2b + 3b| at the chosen point: grad = 5 * y/|y|, so |grad| = 5
    assert torch.isclose(b.grad.norm().cpu(), torch.tensor(5.0))
