"""Grouped ReLU-Conv-BN operations (ops/convbn.py group_relu_conv_bn: one GEMM over the
concatenated weights, per-operation BatchNorm outputs) against fp64 references, and the
AmoebaNet cells that use them against the ungrouped cells."""
import copy

import pytest
import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext, convbn

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert _ext.available(), _ext.load_error()


def rel_err(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


@pytest.fixture(params=[None, (9, 4)], ids=['tuned', 'cfg9-split4'])
def plan(request):
    """Tuned plans, and a forced split-K plan (on 7^2 planes: the partials reduced,
    normalised and their statistics taken by one launch, launch_split_bn_small)."""
    if request.param is not None:
        torch.ops.tgpipe.conv_gemm_force_cfg(*request.param)
    yield request.param
    torch.ops.tgpipe.conv_gemm_force_cfg(-1)


@pytest.mark.parametrize('shape', [(6, 64, 14, (16, 64, 16)), (4, 256, 7, (64, 256, 64)),
                                   (3, 32, 28, (8, 48))], ids=['14x14', '7x7-split', 'two'])
@pytest.mark.parametrize('unused', [False, True], ids=['all-used', 'one-unused'])
def test_grouped_ops_match_fp64(shape, unused, plan):
    n, ci, hw, cos = shape
    torch.manual_seed(0)
    triplets = []
    for co in cos:
        conv = nn.Conv2d(ci, co, 1, bias=False).cuda()
        bn = nn.BatchNorm2d(co).cuda()
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        triplets.append((True, conv, bn))
    refs = [(copy.deepcopy(c).double(), copy.deepcopy(b).double()) for _, c, b in triplets]
    x = torch.randn(n, ci, hw, hw, device='cuda', requires_grad=True)
    x64 = x.detach().double().requires_grad_(True)
    assert convbn.groupable(x, triplets)
    ys = convbn.group_relu_conv_bn(x, triplets, convbn._GroupCache())
    y64s = [b(c(F.relu(x64))) for c, b in refs]
    loss = 0
    loss64 = 0
    torch.manual_seed(1)
    for k, (y, y64) in enumerate(zip(ys, y64s)):
        assert y.shape == y64.shape and y.is_contiguous()
        assert rel_err(y, y64) < 1e-5
        if unused and k == 1:
            continue
        g = torch.randn_like(y)
        loss = loss + (y * g).sum()
        loss64 = loss64 + (y64 * g.double()).sum()
    loss.backward()
    loss64.backward()
    assert rel_err(x.grad, x64.grad) < 1e-5
    for k, ((_, conv, bn), (c64, b64)) in enumerate(zip(triplets, refs)):
        if unused and k == 1:
            # no gradient reached this operation: zero affine gradients (autograd would
            # leave them None; the fused op writes zeros) and a zero weight gradient
            for p in (conv.weight, bn.weight, bn.bias):
                assert p.grad is None or not p.grad.any()
        else:
            assert rel_err(conv.weight.grad, c64.weight.grad) < 1e-5
            assert rel_err(bn.weight.grad, b64.weight.grad) < 1e-5
            assert rel_err(bn.bias.grad, b64.bias.grad) < 1e-5
        assert rel_err(bn.running_mean, b64.running_mean) < 1e-5
        assert rel_err(bn.running_var, b64.running_var) < 1e-6
        assert bn.num_batches_tracked.item() == 1


@pytest.mark.parametrize('cell_streams', [False, True])
def test_grouped_cells_match_ungrouped(cell_streams, monkeypatch):
    """Tiny AmoebaNet-D through PipelineStage: the normal cells' grouped first triplets give
    the ungrouped model's losses, gradients and BatchNorm buffers, step after step."""
    from torchgpipe_amd.models import amoebanetd
    from torchgpipe_amd.models.amoebanet import set_cell_streams
    from torchgpipe_amd.parallel import PipelineStage
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=64)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    if cell_streams:
        set_cell_streams(a, True)
        set_cell_streams(b, True)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last')
    gen = torch.Generator(device=dev).manual_seed(5)
    used = []
    orig = convbn.group_relu_conv_bn

    def spy(*args, **kwargs):
        used.append(1)
        return orig(*args, **kwargs)

    import torchgpipe_amd.models.amoebanet as amoeba
    for k in range(3):
        x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
        y = torch.randint(10, (8,), device=dev, generator=gen)
        for p in list(sa.parameters()) + list(sb.parameters()):
            p.grad = None
        monkeypatch.setattr(convbn, '_GROUP_ENABLED', False)
        la = sa.train_step(x, y, F.cross_entropy)
        monkeypatch.setattr(convbn, '_GROUP_ENABLED', True)
        monkeypatch.setattr(amoeba, 'group_relu_conv_bn', spy)
        lb = sb.train_step(x, y, F.cross_entropy)
        monkeypatch.setattr(amoeba, 'group_relu_conv_bn', orig)
        torch.cuda.synchronize()
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
            assert pb.grad is not None, name
            scale = pa.grad.abs().max().item() + 1e-12
            torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-4, atol=1e-5 * scale,
                                       msg=f'{name} step {k}')
    for (name, ba), bb in zip(a.named_buffers(), b.buffers()):
        torch.testing.assert_close(bb, ba, rtol=1e-4, atol=1e-5, msg=name)
    assert used, 'the grouped op never ran'
