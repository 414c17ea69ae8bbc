"""U-Net resolution-change kernels (csrc/unet_ops.hip) vs PyTorch fp64."""
import pytest
import torch
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext
from torchgpipe_amd.ops.unet_ops import MaxPool2x2, up2x_cat

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    _ext.require()


@pytest.mark.parametrize('shape', [(2, 3, 5, 7, 4), (4, 64, 12, 12, 32), (1, 1, 1, 1, 1)])
def test_up2x_cat_matches_fp64(shape):
    n, c1, h, w, c2 = shape
    torch.manual_seed(0)
    x = torch.randn(n, c1, h, w, device='cuda', requires_grad=True)
    skip = torch.randn(n, c2, 2 * h, 2 * w, device='cuda', requires_grad=True)
    out = up2x_cat(x, skip)
    assert out.grad_fn.__class__.__name__.startswith('_Up2xCat')
    x64 = x.detach().double().requires_grad_()
    s64 = skip.detach().double().requires_grad_()
    ref = torch.cat((F.interpolate(x64, scale_factor=2, mode='nearest'), s64), 1)
    torch.testing.assert_close(out.double(), ref, rtol=0, atol=0)
    g = torch.randn_like(out)
    out.backward(g)
    ref.backward(g.double())
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(skip.grad.double(), s64.grad, rtol=0, atol=0)


def test_up2x_cat_odd_skip_falls_back_to_padding():
    x = torch.randn(2, 3, 4, 4, device='cuda')
    skip = torch.randn(2, 2, 9, 8, device='cuda')
    out = up2x_cat(x, skip)
    up = F.pad(F.interpolate(x, scale_factor=2), [0, 0, 0, 1])
    torch.testing.assert_close(out, torch.cat((up, skip), 1))


@pytest.mark.parametrize('hw', [(8, 8), (7, 9), (2, 2), (192, 192)])
def test_maxpool2x2_matches_aten(hw):
    torch.manual_seed(1)
    x = torch.randn(3, 4, *hw, device='cuda')
    x[0, 0, 0, :2] = 1.5   # ties: the first maximum wins
    x[0, 0, 1, :2] = 1.5
    x[1, 1, 0, 0] = float('nan')
    x[2, 2, 1, 1] = float('nan')
    x.requires_grad_(True)
    y = MaxPool2x2()(x)
    assert y.grad_fn.__class__.__name__.startswith('_MaxPool2x2')
    xr = x.detach().clone().requires_grad_(True)
    yr = F.max_pool2d(xr, 2, 2)
    torch.testing.assert_close(y, yr, equal_nan=True)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(x.grad, xr.grad, equal_nan=True)


@pytest.mark.parametrize('hw', [(14, 14), (7, 9)])
def test_maxpool2x2_add_and_channel_sliced_gradient(hw):
    """AmoebaNet's use: pool(x) + add in one pass, and the gradient of a concatenated cell
    output (a channel slice) read in place."""
    torch.manual_seed(2)
    x = torch.randn(3, 8, *hw, device='cuda', requires_grad=True)
    add = torch.randn(3, 8, hw[0] // 2, hw[1] // 2, device='cuda', requires_grad=True)
    other = torch.randn(3, 5, hw[0] // 2, hw[1] // 2, device='cuda', requires_grad=True)
    y = torch.cat([other, MaxPool2x2()(x, add)], 1)
    xr, ar, orr = (t.detach().double().requires_grad_(True) for t in (x, add, other))
    yr = torch.cat([orr, F.max_pool2d(xr, 2, 2) + ar], 1)
    torch.testing.assert_close(y.double(), yr, rtol=1e-6, atol=1e-6)
    g = torch.randn_like(y)
    y.backward(g)
    yr.backward(g.double())
    torch.testing.assert_close(x.grad.double(), xr.grad, rtol=0, atol=0)
    torch.testing.assert_close(add.grad.double(), ar.grad, rtol=0, atol=0)
