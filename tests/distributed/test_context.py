import pytest
import torch

from torchgpipe_amd.distributed import context


def test_put_get_roundtrip():
    with context.worker('w0', 2):
        x = torch.rand(2)
        context.put_forward('w0', 1, x)
        assert context.get_forward('w0', 1) is x
        context.put_backward('w0', 0, x)
        assert context.get_backward('w0', 0) is x
        context.put_target('w0', x)
        assert context.get_target('w0') is x


def test_unknown_context():
    with pytest.raises(KeyError):
        context.get_forward('nobody', 0)


def test_duplicate_registration():
    with context.worker('dup', 1):
        with pytest.raises(RuntimeError, match='worker dup already exists'):
            with context.worker('dup', 1):
                pass


def test_context_is_removed_after_block():
    with context.worker('tmp', 1):
        assert 'tmp' in context.GlobalContext.ctxs
    assert 'tmp' not in context.GlobalContext.ctxs


def test_decorator():
    @context.distributed('deco', 3)
    def train():
        ctx = context.GlobalContext.get_context('deco')
        return len(ctx.forward_channels), len(ctx.backward_channels)

    assert train() == (3, 3)
    assert 'deco' not in context.GlobalContext.ctxs


def test_utils_to_keeps_requires_grad():
    from torchgpipe_amd.distributed.utils import to
    x = torch.rand(2, requires_grad=True)
    y = to(torch.device('cpu'), x)
    assert y.requires_grad and y.grad_fn is None
    a, b = to(torch.device('cpu'), (x, None))
    assert a.requires_grad and b is None
    assert to(torch.device('cpu'), None) is None


def test_get_module_partition():
    from torch import nn
    from torchgpipe_amd.distributed import get_module_partition
    model = nn.Sequential(nn.Linear(1, 1), nn.ReLU(), nn.Linear(1, 2))
    part = get_module_partition(model, 1, [1, 2], None)
    assert len(part) == 2 and part[1] is model[2]
    with pytest.raises(RuntimeError, match='module and balance mismatch'):
        get_module_partition(model, 2, [1, 2], None)
