"""Numerics of the HIP kernels against plain PyTorch fp32 references (GPU only)."""
import time

import pytest
import torch
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext, fused, misc, philox
from torchgpipe_amd.ops import dropout as dropout_ops

pytestmark = pytest.mark.gpu

cuda = torch.device('cuda', 0)


@pytest.fixture(autouse=True)
def need_ext():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert _ext.available(), f'HIP extension must load on a GPU box: {_ext.load_error()!r}'


@pytest.mark.parametrize('n,seed,offset',
                         [(1, 0, 0), (1001, 12345, 4), (4096, 2 ** 40 + 3, 2 ** 33)])
def test_philox_bit_exact(n, seed, offset):
    got = misc.philox_uniform(n, seed, offset, cuda).cpu()
    want = philox.uniform(n, seed, offset)
    assert torch.equal(got, want)


SHAPES = [
    (2, 3, 6, 6),        # S=36   -> GROUP 16
    (3, 5, 12, 12),      # S=144  -> GROUP 64, V1
    (2, 4, 24, 24),      # S=576  -> GROUP 64, V3
    (2, 3, 48, 48),      # S=2304 -> GROUP 64, V9
    (2, 3, 96, 96),      # S=9216 -> GROUP 256
    (2, 2, 192, 192),    # S=36864 -> GROUP 1024
    (2, 3, 7, 7),        # S=49, scalar path
    (1, 2, 230, 230),    # S=52900 > register tile -> streaming path
]


def _reference(x, p, seed, offset, training, eps=1e-5, slope=1e-2):
    x = x.detach().double().requires_grad_(True)
    n, c = x.shape[:2]
    if training:
        scale = fused.plane_scale_reference(n * c, p, seed, offset, x.device).double()
        d = x * scale.view(n, c, 1, 1)
    else:
        d = x
    y = F.leaky_relu(F.instance_norm(d, eps=eps), slope)
    return x, y


@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('training', [True, False])
def test_drop_norm_act_matches_reference(shape, training):
    torch.manual_seed(0)
    x = (torch.randn(shape, device=cuda) * 3 + 1).requires_grad_(True)
    seed, offset = 987654321, 64
    p = 0.3
    y = fused._DropNormAct.apply(x, p, 1e-5, 1e-2, seed, offset, training)
    dy = torch.randn_like(y)
    y.backward(dy)

    xr, yr = _reference(x, p, seed, offset, training)
    yr.backward(dy.double())
    torch.testing.assert_close(y.double(), yr, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(x.grad.double(), xr.grad, rtol=1e-3, atol=1e-4)


def test_drop_norm_act_module_replays_under_tape():
    from torchgpipe_amd.utils.rng import RngTape
    x = torch.randn(4, 8, 24, 24, device=cuda)
    tape = RngTape()
    with tape.recording():
        a = fused.drop_norm_act(x, 0.5, training=True)
    with tape.replaying():
        b = fused.drop_norm_act(x, 0.5, training=True)
    c = fused.drop_norm_act(x, 0.5, training=True)
    assert torch.equal(a, b)
    assert not torch.equal(a, c)


@pytest.mark.parametrize('n', [1, 7, 4096, 100003])
def test_dropout_kernel(n):
    x = torch.randn(n, device=cuda, requires_grad=True)
    seed, offset = 42, 8
    y = dropout_ops._Dropout.apply(x, 0.25, seed, offset)
    want = dropout_ops._reference(x.detach().cpu(), 0.25, seed, offset)
    torch.testing.assert_close(y.detach().cpu(), want)
    y.backward(torch.ones_like(y))
    torch.testing.assert_close(x.grad.cpu(), (want != 0).float() / 0.75)


def test_pack_unpack_roundtrip():
    ts = [torch.randn(3, 5, device=cuda), torch.arange(7, device=cuda),
          torch.randn(2, 2, 2, device=cuda).half()]
    buf = torch.empty(misc.packed_nbytes(ts), dtype=torch.uint8, device=cuda)
    misc.pack(ts, buf)
    outs = [torch.empty_like(t) for t in ts]
    misc.unpack(buf, outs)
    for a, b in zip(ts, outs):
        assert torch.equal(a, b)


def test_spin_kernel_waits():
    torch.cuda.synchronize()
    start = time.perf_counter()
    misc.spin(0.05, cuda)
    torch.cuda.synchronize()
    assert time.perf_counter() - start >= 0.045
