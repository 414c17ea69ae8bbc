import pytest
import torch

from torchgpipe_amd.microbatch import Batch, check, gather, scatter


def test_batch_atomic():
    x = torch.tensor(42)
    b = Batch(x)
    assert b.atomic
    assert b.tensor is x
    with pytest.raises(AttributeError, match='batch is atomic'):
        b.tensors
    assert list(b) == [x]
    assert len(b) == 1
    assert b[0] is x


def test_batch_non_atomic():
    x, y = torch.tensor(42), torch.tensor(21)
    b = Batch((x, y))
    assert not b.atomic
    with pytest.raises(AttributeError, match='not atomic batch'):
        b.tensor
    assert list(b) == [x, y]
    assert len(b) == 2
    assert b[0] is x and b[1] is y


def test_batch_call():
    a = Batch(torch.tensor(42))
    b = Batch((torch.tensor(42), torch.tensor(21)))

    def f(x):
        return x

    assert a.call(f).atomic
    assert not b.call(f).atomic


def test_batch_setitem_by_index():
    a = Batch(torch.tensor(42))
    b = Batch((torch.tensor(42), torch.tensor(21)))
    a[0] = torch.tensor(0)
    b[0] = torch.tensor(0)
    assert a.atomic and a[0].item() == 0
    assert not b.atomic and len(b) == 2 and b[0].item() == 0 and b[1].item() == 21
    with pytest.raises(IndexError, match='atomic batch allows index 0 only'):
        a[1] = torch.tensor(1)


def test_batch_setitem_by_slice():
    a = Batch(torch.tensor(42))
    b = Batch((torch.tensor(42), torch.tensor(21)))
    a[:] = (torch.tensor(0),)
    b[:] = (torch.tensor(0),)
    assert a.atomic and a[0].item() == 0
    assert not b.atomic and len(b) == 1 and b[0].item() == 0
    with pytest.raises(NotImplementedError, match='only slice'):
        a[1:] = (torch.tensor(0),)
    with pytest.raises(IndexError, match='cannot be replaced with multiple tensors'):
        a[:] = (torch.tensor(0), torch.tensor(1))


def test_check():
    check(torch.tensor(42))
    check((torch.tensor(4), torch.tensor(2)))
    with pytest.raises(TypeError, match='expected Tensor, but got int'):
        check(42)
    with pytest.raises(TypeError):
        check('str')
    with pytest.raises(TypeError):
        check((torch.tensor(4), 2))


def test_gather_tensors():
    a = torch.zeros(1, 1)
    b = torch.zeros(1, 1)
    out = gather([Batch(a), Batch(b)])
    assert out.size() == (2, 1)


def test_gather_tuples():
    a = (torch.zeros(1, 1), torch.zeros(2, 2))
    b = (torch.zeros(1, 1), torch.zeros(2, 2))
    out = gather([Batch(a), Batch(b)])
    assert isinstance(out, tuple)
    assert out[0].size() == (2, 1)
    assert out[1].size() == (4, 2)


def test_scatter_tensor():
    batches = scatter(torch.zeros(2, 1), chunks=2)
    assert len(batches) == 2
    assert batches[0].tensor.size() == (1, 1)


def test_scatter_tuple():
    batches = scatter((torch.zeros(2, 1), torch.zeros(4, 2)), chunks=2)
    assert len(batches) == 2
    assert batches[0][0].size() == (1, 1)
    assert batches[0][1].size() == (2, 2)


def test_scatter_fewer_chunks_than_requested():
    # Tensor.chunk semantics: 6 rows in 4 chunks -> 3 micro-batches of 2.
    batches = scatter(torch.zeros(6, 1), chunks=4)
    assert [b.tensor.size(0) for b in batches] == [2, 2, 2]


def test_scatter_is_a_view():
    x = torch.zeros(4, 3)
    batches = scatter(x, chunks=2)
    batches[0].tensor[0, 0] = 1
    assert x[0, 0] == 1
