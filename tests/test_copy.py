import pytest
import torch

from torchgpipe_amd.copy import Copy, Wait
from torchgpipe_amd.stream import CPUStream, current_stream, new_stream, use_stream


def _copy_wait(prev_stream, next_stream, cuda_sleep=None):
    device = next_stream.device if hasattr(next_stream, 'device') else torch.device('cpu')
    x = torch.ones(1, device=prev_stream.device if hasattr(prev_stream, 'device') else 'cpu',
                   requires_grad=True)
    y, = Copy.apply(prev_stream, next_stream, x)
    y, = Wait.apply(prev_stream, next_stream, y)
    assert y.device.type == device.type
    with use_stream(next_stream):
        z = y * 2
    z.backward()
    assert x.grad.item() == 2.0


def test_copy_wait_cpu_cpu():
    _copy_wait(CPUStream, CPUStream)


@pytest.mark.gpu
@pytest.mark.parametrize('direction', ['cpu_cuda', 'cuda_cpu', 'cuda_cuda'])
def test_copy_wait_gpu(direction):
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    cpu = CPUStream
    gpu = new_stream(torch.device('cuda'))
    prev, nxt = {'cpu_cuda': (cpu, gpu), 'cuda_cpu': (gpu, cpu),
                 'cuda_cuda': (gpu, new_stream(torch.device('cuda')))}[direction]
    x = torch.ones(4, device='cuda' if direction != 'cpu_cuda' else 'cpu', requires_grad=True)
    y, = Copy.apply(prev, nxt, x)
    y, = Wait.apply(prev, nxt, y)
    (y * 3).sum().backward()
    assert torch.equal(x.grad.cpu(), torch.full((4,), 3.0))


def test_wait_detaches():
    x = torch.ones(1, requires_grad=True)
    y, = Wait.apply(CPUStream, CPUStream, x)
    assert y is not x
    assert y.grad_fn is not None
    _ = current_stream(torch.device('cpu'))


def test_wait_multiple_tensors_share_one_node():
    a = torch.rand(2, requires_grad=True)
    b = torch.rand(3, requires_grad=True)
    a2, b2 = Wait.apply(CPUStream, CPUStream, a, b)
    assert a2.grad_fn is b2.grad_fn
    (a2.sum() + 2 * b2.sum()).backward()
    assert torch.equal(a.grad, torch.ones(2)) and torch.equal(b.grad, torch.full((3,), 2.0))
