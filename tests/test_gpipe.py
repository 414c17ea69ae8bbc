from collections import OrderedDict
from copy import deepcopy
import time
from warnings import catch_warnings

import pytest
import torch
from torch import nn

from torchgpipe_amd import GPipe
from torchgpipe_amd.gpipe import verify_module


def count_nodes(grad_fn, name, seen=None):
    seen = set() if seen is None else seen
    if grad_fn is None or grad_fn in seen:
        return 0
    seen.add(grad_fn)
    if type(grad_fn).__name__ == name:
        return 1
    return sum(count_nodes(g, name, seen) for g, _ in grad_fn.next_functions)


def test_parameters():
    gpipe = GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'], chunks=1)
    assert list(gpipe.parameters())


def test_public_attrs_are_coerced():
    class Str:
        def __init__(self, v):
            self.v = v

        def __str__(self):
            return self.v

    gpipe = GPipe(nn.Sequential(nn.Linear(1, 1)), balance=(1,), devices=('cpu',),
                  chunks=42.000, checkpoint=Str('always'))
    assert gpipe.balance == [1]
    assert gpipe.devices == [torch.device('cpu')]
    assert gpipe.chunks == 42 and isinstance(gpipe.chunks, int)
    assert gpipe.checkpoint == 'always' and isinstance(gpipe.checkpoint, str)


@pytest.mark.parametrize('balance', [[2], [1, 1]])
def test_sequential_like(balance):
    a, b = nn.Linear(1, 1), nn.Linear(1, 1)
    model = GPipe(nn.Sequential(a, b), balance, devices=['cpu', 'cpu'])
    assert len(model) == 2
    assert list(model) == [a, b]
    assert model[0] is a and model[1] is b
    assert model[-1] is b and model[-2] is a
    with pytest.raises(IndexError):
        model[2]


@pytest.mark.parametrize('balance', [[1], [3], [0, 2], [-1, 3]])
def test_bad_balance(balance):
    with pytest.raises(ValueError):
        GPipe(nn.Sequential(nn.Linear(1, 1), nn.Linear(1, 1)), balance=balance,
              devices=['cpu', 'cpu'])


@pytest.mark.parametrize('chunks', [0, -1])
def test_chunks_less_than_1(chunks):
    with pytest.raises(ValueError, match='number of chunks must be positive integer'):
        GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'], chunks=chunks)


def test_too_few_devices():
    model = nn.Sequential(*[nn.Linear(1, 1) for _ in range(4)])
    with pytest.raises(IndexError):
        GPipe(model, balance=[1, 1, 1, 1], devices=['cpu'])


@pytest.mark.parametrize('batch', [7, 2])
def test_batch_size_indivisible_or_small(batch):
    model = GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'], chunks=4)
    with catch_warnings(record=True) as record:
        model(torch.rand(batch, 1))
    assert not record


def test_checkpoint_modes_count_checkpoint_nodes():
    model = nn.Sequential(nn.Linear(1, 1))
    x = torch.rand(2, 1)
    outputs = {mode: GPipe(model, balance=[1], devices=['cpu'], chunks=2, checkpoint=mode)(x)
               for mode in ('always', 'except_last', 'never')}
    assert count_nodes(outputs['always'].grad_fn, 'CheckpointBackward') == 2
    assert count_nodes(outputs['except_last'].grad_fn, 'CheckpointBackward') == 1
    assert count_nodes(outputs['never'].grad_fn, 'CheckpointBackward') == 0


def test_checkpoint_mode_invalid():
    with pytest.raises(ValueError,
                       match="checkpoint is not one of 'always', 'except_last', or 'never'"):
        GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'], chunks=2,
              checkpoint='INVALID_CHECKPOINT')


def test_checkpoint_mode_when_chunks_1():
    for mode in ('except_last', 'always', 'never'):
        GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'], chunks=1,
              checkpoint=mode)


def test_checkpoint_disabled_in_eval():
    model = GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'], chunks=2)
    x = torch.rand(2, 1)
    model.train()
    out = model(x)
    assert count_nodes(out.grad_fn, 'CheckpointBackward')
    assert count_nodes(out.grad_fn, 'RecomputeBackward')
    model.eval()
    out = model(x)
    assert not count_nodes(out.grad_fn, 'CheckpointBackward')
    assert not count_nodes(out.grad_fn, 'RecomputeBackward')


def test_no_grad_propagates_to_workers():
    model = GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'], chunks=2)
    seen = []
    model.partitions[0].register_forward_hook(lambda m, i, o: seen.append(o))
    with torch.no_grad():
        model(torch.rand(2, 1))
    assert seen and all(o.grad_fn is None for o in seen)


def test_exception_propagates():
    class Boom(Exception):
        pass

    class Raise(nn.Module):
        def forward(self, *_):
            raise Boom()

    model = GPipe(nn.Sequential(Raise()), balance=[1], devices=['cpu'], chunks=1)
    with pytest.raises(Boom):
        model(torch.rand(1))


def test_exception_early_stop_asap():
    class Boom(Exception):
        pass

    class Pass(nn.Module):
        def forward(self, x):
            return x

    counter = 0

    class Counter(nn.Module):
        def forward(self, x):
            time.sleep(0.1)
            nonlocal counter
            counter += 1
            return x

    class Raise(nn.Module):
        def forward(self, x):
            raise Boom()

    model = GPipe(nn.Sequential(Pass(), Pass(), Counter(), Raise()), [1, 1, 1, 1],
                  devices=['cpu'] * 4, chunks=3)
    with pytest.raises(Boom):
        model(torch.rand(3))
    # The clock cycle that raised still drains, but no later cycle is scheduled.
    assert counter == 2


def test_input_pair():
    class Two(nn.Module):
        def __init__(self):
            super().__init__()
            self.fa = nn.Linear(1, 1)
            self.fb = nn.Linear(1, 1)

        def forward(self, ab):
            a, b = ab
            return self.fa(a), self.fb(b)

    model = GPipe(nn.Sequential(Two()), balance=[1], devices=['cpu'], chunks=2)
    a = torch.rand(10, 1, requires_grad=True)
    b = torch.rand(10, 1, requires_grad=True)
    ao, bo = model((a, b))
    (ao + bo).mean().backward()
    assert a.grad is not None and b.grad is not None


def test_input_singleton_tuple():
    class One(nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = nn.Linear(1, 1)

        def forward(self, only):
            a, = only
            return (self.fc(a),)

    model = GPipe(nn.Sequential(One()), balance=[1], devices=['cpu'], chunks=2)
    a = torch.rand(10, 1, requires_grad=True)
    out, = model((a,))
    out.mean().backward()
    assert all(p.grad is not None for p in model.parameters())
    assert a.grad is not None


def test_input_varargs():
    model = GPipe(nn.Sequential(nn.Linear(1, 1)), balance=[1], devices=['cpu'])
    with pytest.raises(TypeError):
        model(torch.rand(1), torch.rand(1))


def test_non_tensor():
    class NonTensor(nn.Module):
        def forward(self, _):
            return 'hello'

    model = GPipe(nn.Sequential(NonTensor()), balance=[1], devices=['cpu'])
    with pytest.raises(TypeError):
        model(torch.rand(1))
    with pytest.raises(TypeError):
        model('hello')


def test_non_tensor_tuple():
    class NonTensorTuple(nn.Module):
        def forward(self, x):
            return (x, 'hello')

    model = GPipe(nn.Sequential(NonTensorTuple()), balance=[1], devices=['cpu'])
    with pytest.raises(TypeError):
        model(torch.rand(1))
    with pytest.raises(TypeError):
        model((torch.rand(1), 'hello'))


@pytest.mark.parametrize('checkpoint', ['never', 'always', 'except_last'])
def test_deferred_batch_norm(checkpoint):
    bn = nn.BatchNorm2d(3)
    gpipe = GPipe(nn.Sequential(deepcopy(bn)), balance=[1], devices=['cpu'], chunks=2,
                  checkpoint=checkpoint, deferred_batch_norm=True)
    x = torch.rand(4, 3, 10, 10)
    gpipe(x).mean().backward()
    bn(x).mean().backward()
    torch.testing.assert_close(gpipe[0].running_mean, bn.running_mean, atol=1e-4, rtol=0)
    torch.testing.assert_close(gpipe[0].running_var, bn.running_var, atol=1e-4, rtol=0)


@pytest.mark.parametrize('checkpoint', ['never', 'always'])
def test_deferred_batch_norm_params(checkpoint):
    bn = nn.BatchNorm2d(3)
    gpipe = GPipe(nn.Sequential(deepcopy(bn)), balance=[1], devices=['cpu'], chunks=1,
                  checkpoint=checkpoint, deferred_batch_norm=True)
    x = torch.rand(4, 3, 10, 10)
    gpipe(x).mean().backward()
    bn(x).mean().backward()
    torch.testing.assert_close(gpipe[0].weight.grad, bn.weight.grad, atol=1e-4, rtol=0)
    torch.testing.assert_close(gpipe[0].bias.grad, bn.bias.grad, atol=1e-4, rtol=0)


def test_extra_devices_are_dropped():
    model = GPipe(nn.Sequential(*[nn.Linear(1, 1) for _ in range(3)]), [1, 1, 1],
                  devices=['cpu'] * 5)
    assert model.devices == [torch.device('cpu')] * 3


def test_partitions_and_state_dict_format():
    model = GPipe(nn.Sequential(nn.Linear(1, 1), nn.Linear(1, 1)), [1, 1], devices=['cpu'] * 2)
    assert isinstance(model.partitions, nn.ModuleList)
    assert all(isinstance(p, nn.Sequential) for p in model.partitions)
    keys = set(model.state_dict())
    assert {'partitions.0.0.weight', 'partitions.0.0.bias',
            'partitions.1.1.weight', 'partitions.1.1.bias'} == keys


def test_deny_moving():
    model = GPipe(nn.Sequential(nn.Linear(1, 1), nn.Linear(1, 1)), [1, 1], devices=['cpu'] * 2)
    for call in (lambda: model.cuda(), lambda: model.cpu(),
                 lambda: model.to(torch.device('cuda')), lambda: model.to(0),
                 lambda: model.to('cuda'), lambda: model.to(device=0),
                 lambda: model.to(torch.rand(1)), lambda: model.to(tensor=torch.rand(1))):
        with pytest.raises(TypeError):
            call()
    model.half()
    model.to(torch.double)
    model.to(dtype=torch.float)


def test_empty_module():
    model = GPipe(nn.Sequential(), [])
    assert model(torch.tensor(42)) == torch.tensor(42)
    assert model((torch.tensor(42),)) == (torch.tensor(42),)
    with pytest.raises(TypeError):
        model(42)


def test_named_children():
    model = GPipe(nn.Sequential(OrderedDict([('a', nn.Linear(1, 1)), ('b', nn.Linear(1, 1))])),
                  [1, 1], devices=['cpu'] * 2)
    names = {n for n, _ in model.named_modules()}
    assert 'partitions.0.a' in names and 'partitions.1.b' in names
    with pytest.raises(AttributeError):
        model.a


def test_recommend_auto_balance():
    with pytest.raises(ValueError, match='torchgpipe.balance'):
        GPipe(nn.Sequential())
    with pytest.raises(ValueError, match='torchgpipe_amd.balance'):
        GPipe(nn.Sequential(), [1])
    with pytest.raises(ValueError, match='torchgpipe_amd.balance'):
        GPipe(nn.Sequential(nn.Linear(1, 1), nn.Linear(1, 1)), [1])


def test_verify_module_non_sequential():
    with pytest.raises(TypeError, match='module must be nn.Sequential to be partitioned'):
        verify_module(nn.Module())


def test_verify_module_duplicate_children():
    conv = nn.Conv2d(3, 3, 1)
    with pytest.raises(ValueError, match='module with duplicate children is not supported'):
        verify_module(nn.Sequential(conv, conv))


def test_verify_module_duplicate_parameters_in_distinct_children():
    class Wrap(nn.Module):
        def __init__(self, m):
            super().__init__()
            self.m = m

    conv = nn.Conv2d(3, 3, 1)
    with pytest.raises(ValueError, match='module with duplicate parameters in '
                                         'distinct children is not supported'):
        verify_module(nn.Sequential(Wrap(conv), Wrap(conv)))


def test_repeated_forward_reuses_workers():
    model = GPipe(nn.Sequential(nn.Linear(2, 2), nn.Linear(2, 2)), [1, 1], devices=['cpu'] * 2,
                  chunks=2)
    for _ in range(3):
        model(torch.rand(4, 2)).sum().backward()
    # One persistent thread per distinct device.
    assert len(model._workers._threads) == 1
