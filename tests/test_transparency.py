import copy

import pytest
import torch
from torch import nn

from torchgpipe_amd import GPipe


@pytest.mark.parametrize('checkpoint', ['always', 'except_last', 'never'])
def test_simple_linears(checkpoint):
    def sum_grad(parameters):
        return sum(p.grad.sum() for p in parameters if p.grad is not None)

    def zero_grad(parameters):
        for p in parameters:
            p.grad = None

    inputs = torch.rand(8, 1)
    model = nn.Sequential(nn.Linear(1, 2), nn.Linear(2, 4), nn.Linear(4, 2), nn.Linear(2, 1))

    outputs = model(inputs)
    outputs.mean().backward()
    grad_without_gpipe = sum_grad(model.parameters())
    zero_grad(model.parameters())

    model = GPipe(model, [2, 2], devices=['cpu', 'cpu'], chunks=4, checkpoint=checkpoint)
    outputs = model(inputs)
    outputs.mean().backward()
    grad_with_gpipe = sum_grad(model.parameters())
    assert torch.allclose(grad_with_gpipe, grad_without_gpipe)


@pytest.mark.parametrize('checkpoint', ['always', 'except_last', 'never'])
def test_dropout_model_matches_per_microbatch_reference(checkpoint):
    # With dropout, GPipe must equal running the plain model micro-batch by
    # micro-batch with the same RNG stream (recomputation replays the RNG).
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(4, 8), nn.Dropout(0.5), nn.Linear(8, 8), nn.ReLU(),
                          nn.Dropout(0.3), nn.Linear(8, 1))
    ref = copy.deepcopy(model)
    x = torch.rand(8, 4)

    gpipe = GPipe(model, [3, 3], devices=['cpu', 'cpu'], chunks=2, checkpoint=checkpoint)
    torch.manual_seed(7)
    gpipe(x).sum().backward()

    torch.manual_seed(7)
    # Forward order of the single-threaded CPU pipeline: (0,0),(1,0),(0,1),(1,1).
    a0 = ref[:3](x[:4])
    a1 = ref[:3](x[4:])
    y0 = ref[3:](a0)
    y1 = ref[3:](a1)
    torch.cat([y0, y1]).sum().backward()
    for p, q in zip(gpipe.parameters(), ref.parameters()):
        torch.testing.assert_close(p.grad, q.grad)
