from functools import partial

import pytest
import torch
from torch import nn
import torch.cuda

from torchgpipe_amd.checkpoint import (Checkpointing, checkpoint, is_checkpointing,
                                       is_recomputing)
from torchgpipe_amd.dependency import fork, join
from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.utils.rng import RngTape, philox_pair

devices = ['cpu']
if torch.cuda.is_available():
    devices.append('cuda')


@pytest.mark.parametrize('device', devices)
def test_serial_checkpoints(device):
    # Two checkpoints chained by a phony edge: b's recomputation and backward
    # must both finish before a is recomputed (pytorch/pytorch#18568 scenario).
    events = []

    class Log(torch.autograd.Function):
        @staticmethod
        def forward(ctx, name, x):
            ctx.name = name
            events.append(f'{name}:forward')
            return x.detach()

        @staticmethod
        def backward(ctx, grad_output):
            events.append(f'{ctx.name}:backward')
            return None, grad_output

    a = torch.rand(1, device=device, requires_grad=True)
    b = torch.rand(1, device=device, requires_grad=True)
    _ = a + 1 + 2 + 3 + 4 + 5  # bump the autograd sequence number

    a = checkpoint(partial(Log.apply, 'a'), a)
    a, phony = fork(a)
    b = join(b, phony)
    b = checkpoint(partial(Log.apply, 'b'), b)
    torch.cat((a, b)).sum().backward()

    assert events == ['a:forward', 'b:forward',
                      'b:forward', 'b:backward',
                      'a:forward', 'a:backward']


def test_not_requires_grad():
    x = Batch(torch.rand(1, requires_grad=False))
    assert not x[0].requires_grad

    def f(x):
        return x * 2

    chk = Checkpointing(f, x)
    x = chk.checkpoint()
    assert x[0].requires_grad
    chk.recompute(x)
    assert x[0].requires_grad
    x.tensor.backward()


def test_not_requires_grad_with_parameter():
    x = torch.rand(1, requires_grad=False)
    a = torch.rand(1, requires_grad=True)

    def f(x):
        return x * a

    y = checkpoint(f, x)
    y.backward()
    assert a.grad is not None


@pytest.mark.parametrize('device', devices)
def test_random_in_checkpoint(device):
    dropout = nn.Dropout(p=0.5)
    torch.manual_seed(0)
    x = torch.randn(3, 3, device=device, requires_grad=True)
    y = dropout(x)
    y.norm().backward()

    torch.manual_seed(0)
    chk_x = torch.randn(3, 3, device=device, requires_grad=True)
    chk_y = checkpoint(dropout, chk_x)
    chk_y.norm().backward()

    assert torch.allclose(x.grad, chk_x.grad)


def test_framework_rng_replays_through_tape():
    # The framework's Philox (seed, offset) pairs are recorded while
    # checkpointing and handed back verbatim during recomputation.
    drawn = []

    def f(x):
        drawn.append(philox_pair(x.device, 16))
        return x * 2

    x = torch.rand(2, requires_grad=True)
    y = checkpoint(f, x)
    y.sum().backward()
    assert len(drawn) == 2 and drawn[0] == drawn[1]


def test_rng_tape_exhaustion_is_an_error():
    tape = RngTape()
    with tape.recording():
        philox_pair(torch.device('cpu'), 4)
    with tape.replaying():
        philox_pair(torch.device('cpu'), 4)
        with pytest.raises(RuntimeError, match='exhausted'):
            philox_pair(torch.device('cpu'), 4)


def test_detect_checkpointing_recomputing():
    logs = []

    class Detect(nn.Module):
        def forward(self, input):
            logs.append((is_checkpointing(), is_recomputing()))
            return input

    model = Detect()
    input = torch.rand(1, requires_grad=True)
    output = checkpoint(model, input)
    output.backward()
    assert logs == [(True, False), (False, True)]


def test_detect_checkpointing_recomputing_without_checkpoint():
    logs = []

    class Detect(nn.Module):
        def forward(self, input):
            logs.append((is_checkpointing(), is_recomputing()))
            return input

    model = Detect()
    input = torch.rand(1, requires_grad=True)
    output = model(input)
    output.backward()
    assert logs == [(False, False)]


def test_non_grad_output():
    class ForkNonGrad(nn.Module):
        def forward(self, input):
            return (input * 2, torch.rand(1))

    model = ForkNonGrad()
    input = torch.rand(1, requires_grad=True)
    output = checkpoint(model, input)
    output[0].backward()


def test_recompute_now_precedes_gradient():
    # Explicitly scheduled pipelines recompute eagerly; Checkpoint.backward must
    # then use the precomputed graph rather than recomputing again.
    calls = []

    def f(x):
        calls.append(is_recomputing())
        return x.sin()

    x = torch.rand(4, requires_grad=True)
    chk = Checkpointing(f, Batch(x))
    out = chk.checkpoint()
    chk.recompute_now()
    out.tensor.sum().backward()
    assert calls == [False, True]
    torch.testing.assert_close(x.grad, x.detach().cos())


def test_zoo_dropout2d_replays_from_tape_without_touching_global_rng():
    """Verdict r1 #6c: the model zoo's Dropout2d draws Philox pairs from the cell's tape, so
    'always' and 'never' give identical gradients and recompute leaves torch's RNG alone."""
    from torchgpipe_amd import GPipe
    from torchgpipe_amd.ops.dropout import Dropout2d
    grads = {}
    for mode in ('never', 'always'):
        torch.manual_seed(0)
        model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), Dropout2d(0.5),
                              nn.Conv2d(8, 8, 3, padding=1), Dropout2d(0.5))
        gpipe = GPipe(model, [2, 2], devices=['cpu', 'cpu'], chunks=2, checkpoint=mode)
        x = torch.rand(4, 3, 8, 8)
        torch.manual_seed(123)
        out = gpipe(x)
        state = torch.get_rng_state()
        out.sum().backward()
        # backward (with recomputation under 'always') must not have moved the generator
        assert torch.equal(state, torch.get_rng_state())
        grads[mode] = [p.grad.clone() for p in gpipe.parameters()]
    for a, b in zip(grads['never'], grads['always']):
        assert torch.equal(a, b)


@pytest.mark.parametrize('where', ['gpipe', 'convert'])
def test_user_dropout_on_the_philox_tape(where):
    """GPipe(philox_dropout=True): the user's nn.Dropout / nn.Dropout2d layers draw Philox
    pairs replayed from the checkpoint tape -- 'always' equals 'never' exactly and the
    backward's recomputation leaves torch's generator alone."""
    from torchgpipe_amd import GPipe
    from torchgpipe_amd.ops.dropout import Dropout, Dropout2d, convert_dropout
    grads = {}
    for mode in ('never', 'always'):
        torch.manual_seed(0)
        model = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.Dropout2d(0.5),
                              nn.Sequential(nn.Conv2d(8, 8, 3, padding=1), nn.Dropout(0.3)))
        if where == 'convert':
            convert_dropout(model)
        assert isinstance(model[1], Dropout2d) == (where == 'convert')
        gpipe = GPipe(model, [2, 1], devices=['cpu', 'cpu'], chunks=2, checkpoint=mode,
                      philox_dropout=True)
        assert isinstance(gpipe.partitions[0][1], Dropout2d)
        assert isinstance(gpipe.partitions[1][0][1], Dropout)
        x = torch.rand(4, 3, 8, 8)
        torch.manual_seed(123)
        out = gpipe(x)
        state = torch.get_rng_state()
        out.sum().backward()
        assert torch.equal(state, torch.get_rng_state())
        grads[mode] = [p.grad.clone() for p in gpipe.parameters()]
    for a, b in zip(grads['never'], grads['always']):
        assert torch.equal(a, b)


def test_inplace_change_of_a_checkpointed_input_is_an_error():
    """The Checkpoint node keeps its inputs outside autograd's saved tensors (so a pipeline
    can release them early): the recomputation checks their version counters itself, so
    an in-place change between forward and recomputation fails loudly instead of
    recomputing from the changed value."""
    x = torch.randn(4, 3)
    lin = nn.Linear(3, 2)
    chk = Checkpointing(lin, Batch(x))
    out = chk.checkpoint()
    x.add_(1.0)
    with pytest.raises(RuntimeError, match='inplace'):
        chk.recompute_now()
    del out
