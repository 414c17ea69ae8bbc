"""Backward-data of fused ReLU-Conv-BN operations on the library convolution + ReLU mask
(csrc/convbn.cpp lib_dgrad, chosen per geometry by timing) against the implicit GEMM and an
fp64 reference."""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

from torchgpipe_amd.ops import _ext
from torchgpipe_amd.ops.convbn import fusable, relu_conv_bn

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert _ext.available(), _ext.load_error()


def rel_err(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


CASES = [  # x, out channels, kernel, stride, padding
    ((6, 32, 56, 56), 32, (3, 3), 2, (1, 1)),
    ((6, 256, 28, 28), 128, (1, 1), 2, (0, 0)),
    ((8, 1024, 7, 7), 1024, (1, 1), 1, (0, 0)),
    ((8, 64, 7, 7), 64, (1, 7), 1, (0, 3)),
]


@pytest.mark.parametrize('case', CASES, ids=['3x3s2', '1x1s2', '1x1@7', '1x7@7'])
@pytest.mark.parametrize('mode', [0, 1], ids=['gemm', 'library'])
def test_backward_data_paths_match_fp64(case, mode):
    xs, co, k, s, pad = case
    torch.manual_seed(0)
    conv = nn.Conv2d(xs[1], co, k, stride=s, padding=pad, bias=False).cuda()
    bn = nn.BatchNorm2d(co).cuda()
    x = torch.randn(*xs, device='cuda', requires_grad=True)
    assert fusable(x, [conv], bn)
    torch.ops.tgpipe.lib_dgrad_force(mode)
    try:
        y = relu_conv_bn(x, [(conv, 0)], bn)
        dy = torch.randn_like(y)
        y.backward(dy)
    finally:
        torch.ops.tgpipe.lib_dgrad_force(-1)
    x64 = x.detach().double().requires_grad_(True)
    ref = F.batch_norm(F.conv2d(F.relu(x64), conv.weight.double(), stride=s, padding=pad),
                       None, None, bn.weight.double(), bn.bias.double(), True, 0.0, bn.eps)
    ref.backward(dy.double())
    assert rel_err(x.grad, x64.grad) < 2e-5


def test_measured_choice_is_recorded_per_geometry():
    """An unforced eager call decides once per geometry (lib_dgrad_export lists the
    geometries that went to the library); the gradient is the same either way."""
    torch.manual_seed(0)
    conv = nn.Conv2d(32, 32, 3, stride=2, padding=1, bias=False).cuda()
    bn = nn.BatchNorm2d(32).cuda()
    x = torch.randn(6, 32, 56, 56, device='cuda', requires_grad=True)
    r = torch.randn(6, 32, 28, 28, device='cuda')  # (a BatchNorm output's square sum is
    grads = []                                      # constant: no gradient to compare)
    for _ in range(2):
        x.grad = None
        (relu_conv_bn(x, [(conv, 0)], bn) * r).sum().backward()
        grads.append(x.grad.clone())
    table = torch.ops.tgpipe.lib_dgrad_export()
    assert isinstance(table, str)
    for line in table.splitlines():
        assert len(line.split()) == 11
    assert rel_err(grads[1], grads[0]) < 1e-5
