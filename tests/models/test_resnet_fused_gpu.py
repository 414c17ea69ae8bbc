"""Fused ResNet layers (ops/fusion.py: ConvBN2d -> BatchNormAct2d -> ReLU runs) against fp64
``nn`` references of the same layers, and the fused ResNet-50 against the plain model."""
import copy

import pytest
import torch
from torch import nn

from torchgpipe_amd.ops import _ext
from torchgpipe_amd.ops.fusion import BatchNormAct2d, ConvBN2d, ReLU, relink

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert _ext.available(), _ext.load_error()


def rel_err(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


# (n, ci, hw, co, kernel, stride, padding)
CASES = [
    (4, 64, 28, 96, 1, 1, 0),     # 1x1: implicit GEMM, statistics in the epilogue
    (4, 64, 28, 128, 1, 2, 0),    # strided 1x1 (downsample): MIOpen + native BN
    (4, 64, 28, 64, 3, 1, 1),     # 3x3 stride 1: Winograd F(4x4) + native BN(+ReLU)
    (4, 256, 14, 256, 3, 1, 1),   # 3x3 stride 1, >= 256 channels: batched-GEMM Winograd
    (4, 32, 28, 32, 3, 2, 1),     # 3x3 stride 2: MIOpen + native BN(+ReLU)
    (2, 3, 64, 64, 7, 2, 3),      # the stem 7x7 stride 2: MIOpen + native BN(+ReLU)
    (4, 512, 7, 512, 1, 1, 0),    # 7x7 planes: split reduction, fused split statistics
    # the strided geometries shipped on the fused native op (ops/fusion.py STRIDED_FUSED):
    # implicit-GEMM forward + stride-phase backward-data
    (2, 128, 56, 128, 3, 2, 1),
    (2, 256, 56, 512, 1, 2, 0),
    (2, 512, 14, 512, 3, 2, 1),
    (2, 3, 224, 64, 7, 2, 3),     # (round 6: the stem and the 28^2 / 14^2 downsamples)
    (2, 512, 28, 1024, 1, 2, 0),
    (2, 1024, 14, 2048, 1, 2, 0),
]


@pytest.mark.parametrize('relu', [True, False])
@pytest.mark.parametrize('case', CASES, ids=[f'{c[4]}x{c[4]}s{c[5]}_{c[1]}to{c[3]}@{c[2]}'
                                            for c in CASES])
def test_conv_bn_relu_run_matches_fp64(case, relu):
    n, ci, hw, co, k, stride, pad = case
    torch.manual_seed(0)
    mods = [ConvBN2d(ci, co, k, stride=stride, padding=pad, bias=False), BatchNormAct2d(co)]
    if relu:
        mods.append(ReLU())
    seq = nn.Sequential(*mods).cuda()
    with torch.no_grad():
        seq[1].weight.uniform_(0.5, 1.5)
        seq[1].bias.uniform_(-0.5, 0.5)
    assert relink(seq) == 1
    ref = nn.Sequential(nn.Conv2d(ci, co, k, stride=stride, padding=pad, bias=False),
                        nn.BatchNorm2d(co)).cuda().double()
    ref.load_state_dict(seq.state_dict(), strict=False)
    x = torch.randn(n, ci, hw, hw, device='cuda', requires_grad=True)
    x64 = x.detach().double().requires_grad_(True)
    y = seq(x)
    assert getattr(y, '_tgpipe_bn_done', None) == id(seq[1]), 'the fused path must run'
    y64 = ref(x64)
    if relu:
        # The ReLU in fp64 with the fused forward's own decisions: a value within rounding
        # of zero may fall on the other side in fp64, and each such flip moves a whole
        # gradient element (benchmarks/diag/resnet_fused_diag2.py: 2.9e-6 on the
        # convolution output becomes 6.8e-3 on dz through a handful of flips -- for any
        # fp32 implementation, MIOpen's included).
        y64 = y64 * (y > 0).double()
    assert rel_err(y, y64) < 1e-5
    g = torch.randn_like(y)
    y.backward(g)
    y64.backward(g.double())
    assert rel_err(x.grad, x64.grad) < 2e-5
    for (name, p), q in zip(seq.named_parameters(), ref.parameters()):
        assert rel_err(p.grad, q.grad) < 2e-5, name
    # (the batch mean of a ~zero-mean output is ill-conditioned: the Winograd output's
    # ~1e-6 relative error shows up a few times larger in it)
    assert rel_err(seq[1].running_mean, ref[1].running_mean) < 2e-5
    assert rel_err(seq[1].running_var, ref[1].running_var) < 2e-6
    assert seq[1].num_batches_tracked.item() == 1


def test_unlinked_layers_run_on_their_own():
    """A balance that separates the convolution from its BatchNorm: each layer runs alone
    (implicit-GEMM convolution, native BatchNorm + ReLU) and computes the same function."""
    torch.manual_seed(0)
    full = nn.Sequential(ConvBN2d(32, 48, 1, bias=False), BatchNormAct2d(48), ReLU()).cuda()
    other = copy.deepcopy(full)
    assert relink(full) == 1
    a, b = nn.Sequential(other[0]), nn.Sequential(other[1], other[2])
    assert relink(a) == 0 and relink(b) == 0
    x = torch.randn(4, 32, 14, 14, device='cuda', requires_grad=True)
    x2 = x.detach().clone().requires_grad_(True)
    y_fused = full(x)
    y_split = b(a(x2))
    assert getattr(y_split, '_tgpipe_bn_done', None) is None
    assert rel_err(y_split, y_fused) < 1e-5
    y_fused.square().sum().backward()
    y_split.square().sum().backward()
    assert rel_err(x2.grad, x.grad) < 1e-5
    for p, q in zip(full.parameters(), other.parameters()):
        assert rel_err(q.grad, p.grad) < 1e-5
    assert rel_err(other[1].running_var, full[1].running_var) < 1e-6


def test_fused_resnet50_matches_plain_model():
    """Whole fused ResNet-50 (training mode) and the plain fp32 nn model (MIOpen) against
    the fp64 model with the same weights: the fused model's loss, input gradient, parameter
    gradients and BatchNorm running statistics are as close to fp64 as the plain model's
    (a deep BatchNorm network's gradients are ill-conditioned for any fp32 arithmetic)."""
    from torchgpipe_amd.models.resnet import build_resnet
    torch.manual_seed(0)
    fused = build_resnet([3, 4, 6, 3], num_classes=10, fused=True).cuda()
    plain = build_resnet([3, 4, 6, 3], num_classes=10, fused=False).cuda()
    plain.load_state_dict(fused.state_dict())
    ref = copy.deepcopy(plain).double()
    x = torch.randn(16, 3, 96, 96, device='cuda')
    t = torch.randint(10, (16,), device='cuda')
    res = []
    for model, dt in ((fused, torch.float32), (plain, torch.float32), (ref, torch.float64)):
        xi = x.clone().to(dt).requires_grad_(True)
        loss = nn.functional.cross_entropy(model(xi), t)
        loss.backward()
        res.append((loss.detach(), xi.grad, [p.grad for p in model.parameters()],
                    [b for b in model.buffers() if b.is_floating_point()]))
    (lf, xf, gf, bf), (lp, xp, gp, bp), (l64, x64, g64, b64) = res
    assert rel_err(lf, l64) < 1e-5
    # (through 50 layers of BatchNorm + ReLU the per-layer mask flips of any fp32 forward
    # compound: the plain fp32 model itself is ~1e-3 off fp64 on the deep gradients; the
    # fused model must stay within a small multiple of that)
    assert rel_err(xf, x64) < max(1e-3, 8 * rel_err(xp, x64))
    names = [n for n, _ in fused.named_parameters()]
    for name, a, b, r in zip(names, gf, gp, g64):
        assert a is not None and b is not None and r is not None, name
        assert rel_err(a, r) < max(1e-3, 8 * rel_err(b, r)), name
    for a, b, r in zip(bf, bp, b64):
        assert rel_err(a, r) < max(1e-5, 4 * rel_err(b, r))


@pytest.mark.parametrize('shape', [(4, 256, 14), (2, 1024, 7)], ids=['256@14', '1024@7'])
def test_residual_join_runs_conv3_bn3_add_relu_as_one_op(shape):
    """A bottleneck's conv3, bn3, residual, relu3 (ops/fusion.py pending_join): the join's
    output and every gradient against the fp64 plain bottleneck (ReLU decisions of the
    fused forward)."""
    from torchgpipe_amd.models.resnet import bottleneck
    from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker
    n, c, hw = shape
    torch.manual_seed(0)
    fused = bottleneck(c, c // 4, fused=True).cuda()
    plain = bottleneck(c, c // 4, fused=False).cuda().double()
    plain.load_state_dict(fused.state_dict())
    with torch.no_grad():
        for m in fused.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.weight.uniform_(0.5, 1.5)
                m.bias.uniform_(-0.5, 0.5)
    plain.load_state_dict(fused.state_dict())
    assert relink(fused) == 3
    conv3 = fused.conv3
    assert conv3.__dict__['_tgpipe_link'][2] is not None
    x = torch.randn(n, c, hw, hw, device='cuda').relu().requires_grad_(True)
    x64 = x.detach().double().requires_grad_(True)
    with use_skip_tracker(SkipTracker()):
        y = fused(x)
    with use_skip_tracker(SkipTracker()):
        y64 = plain(x64)
    assert getattr(y, '_tgpipe_relu_done', False)
    # the identity's gradient goes to conv1's backward-data GEMM (GradSink)
    from torchgpipe_amd.ops import fusion
    sink = getattr(x, '_tgpipe_grad_sink', None)
    assert (sink is not None and sink.claimed) or not fusion.GRAD_SINK
    y64 = y64 * (y > 0).double()
    assert rel_err(y, y64) < 1e-5
    g = torch.randn_like(y)
    y.backward(g)
    y64.backward(g.double())
    # relu1 / relu2 decide in fp64 on their own: the plain fp32 bottleneck's error against
    # the same reference sets the scale of what those flips may cost
    plain32 = copy.deepcopy(plain).float()
    x32 = x.detach().clone().requires_grad_(True)
    with use_skip_tracker(SkipTracker()):
        y32 = plain32(x32)
    (y32 * (y > 0).float()).backward(g)
    gate = max(5e-5, 8 * rel_err(x32.grad, x64.grad))
    assert rel_err(x.grad, x64.grad) < gate
    for (name, p), q, r in zip(fused.named_parameters(), plain.parameters(),
                               plain32.parameters()):
        assert rel_err(p.grad, q.grad) < max(5e-5, 8 * rel_err(r.grad, q.grad)), name
    assert rel_err(fused.bn3.running_var, plain.bn3.running_var) < 2e-6


@pytest.mark.parametrize('shape', [(4, 256, 14), (2, 1024, 7), (12, 128, 56)],
                         ids=['vec', 'scalar', 'two-pass'])
def test_join_mask_inside_batchnorm_backward_matches_separate_relu(shape):
    """The residual join's ReLU mask applied inside the BatchNorm backward (the mask from the
    saved output, the masked gradient written for the identity: ``convbn_backward``'s
    ``y_mask``) against the same join computed as Conv-BN, then ``relu(y + identity)`` by
    autograd -- same forward arithmetic, so the same ReLU decisions: every gradient equal.
    14^2: the 16-byte one-pass kernel, 7^2: its scalar loop, 56^2 at 12 images (37.6 k
    values per channel): the two-pass backward after a separate masking pass."""
    from torchgpipe_amd.ops.convbn import relu_conv_bn
    n, c, hw = shape
    torch.manual_seed(3)
    conv = nn.Conv2d(c, c, 1, bias=False).cuda()
    bn = nn.BatchNorm2d(c).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    x = torch.randn(n, c, hw, hw, device='cuda')
    ident = torch.randn(n, c, hw, hw, device='cuda')
    g = torch.randn(n, c, hw, hw, device='cuda')
    xa, ia = x.clone().requires_grad_(True), ident.clone().requires_grad_(True)
    ya = relu_conv_bn(xa, [(conv, 0)], bn, relu=False, add=ia, relu_out=True)
    ya.backward(g)
    xb, ib = x.clone().requires_grad_(True), ident.clone().requires_grad_(True)
    yb = torch.relu(relu_conv_bn(xb, [(conv2, 0)], bn2, relu=False) + ib)
    yb.backward(g)
    torch.testing.assert_close(ya, yb, rtol=0, atol=0)
    for a, b in [(xa.grad, xb.grad), (ia.grad, ib.grad), (conv.weight.grad, conv2.weight.grad),
                 (bn.weight.grad, bn2.weight.grad), (bn.bias.grad, bn2.bias.grad)]:
        torch.testing.assert_close(a, b, rtol=1e-6, atol=1e-6 * (b.abs().max().item() + 1))


def test_native_batchnorm_affine_gradients_accumulate_across_micro_batches():
    """The native BatchNorm(+ReLU) after a Winograd 3x3 (``_BNAct``) adds its gamma / beta
    gradients into ``.grad`` in the kernel (ops/gradacc.py) -- over several backward
    passes (micro-batches) the same sums as autograd's accumulation of the plain layers."""
    torch.manual_seed(0)
    seq = nn.Sequential(ConvBN2d(32, 32, 3, padding=1, bias=False), BatchNormAct2d(32),
                        ReLU()).cuda()
    with torch.no_grad():
        seq[1].weight.uniform_(0.5, 1.5)
        seq[1].bias.uniform_(-0.5, 0.5)
    ref = nn.Sequential(nn.Conv2d(32, 32, 3, padding=1, bias=False), nn.BatchNorm2d(32),
                        nn.ReLU()).cuda().double()
    ref.load_state_dict(seq.state_dict(), strict=False)
    assert relink(seq) == 1
    for k in range(3):
        x = torch.randn(4, 32, 14, 14, device='cuda')
        y = seq(x)
        assert getattr(y, '_tgpipe_bn_done', None) == id(seq[1])
        y64 = ref(x.double()) * (y > 0).double()
        g = torch.randn_like(y)
        y.backward(g)
        y64.backward(g.double())
        for (name, p), q in zip(seq.named_parameters(), ref.parameters()):
            assert rel_err(p.grad, q.grad) < 2e-5, (k, name)
