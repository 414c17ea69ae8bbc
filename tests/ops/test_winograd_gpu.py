"""Winograd F(4x4,3x3) / F(2x2,3x3) MFMA convolutions vs an fp64 PyTorch convolution (GPU only)."""
import copy

import pytest
import torch
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext
from torchgpipe_amd.ops.conv import WinogradConv2d, winograd_conv2d

pytestmark = pytest.mark.gpu
cuda = torch.device('cuda', 0)


@pytest.fixture(autouse=True)
def need_ext():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert _ext.available(), f'HIP extension must load on a GPU box: {_ext.load_error()!r}'


SHAPES = [  # (N, C, K, H, W)
    (2, 3, 64, 16, 16),     # C not a multiple of the 8-channel chunk (U-Net input conv)
    (2, 64, 64, 24, 24),
    (1, 5, 70, 7, 9),       # odd H/W, K not a multiple of 64
    (3, 128, 256, 6, 6),
    (2, 256, 128, 12, 12),
    (1, 16, 8, 1, 1),
    (4, 32, 32, 33, 2),
    (2, 64, 96, 40, 40),    # fused F(4x4) forward / weight gradient
    (2, 512, 640, 12, 12),  # non-fused F(4x4) forward, backward-data and weight gradient
    (2, 512, 512, 6, 6),    # 6x6 with >= 512 channels: F(4x4) non-fused at <= 24 images
]


def _ref(x, w, b=None):
    return F.conv2d(x.double(), w.double(), None if b is None else b.double(), padding=1)


@pytest.mark.parametrize('shape', SHAPES)
@pytest.mark.parametrize('bias', [False, True])
def test_forward_backward_match_conv2d(shape, bias):
    n, c, k, h, w = shape
    torch.manual_seed(0)
    x = torch.randn(n, c, h, w, device=cuda, requires_grad=True)
    conv = WinogradConv2d(c, k, 3, padding=1, bias=bias).to(cuda)
    y = conv(x)
    dy = torch.randn_like(y)
    y.backward(dy)

    xr = x.detach().double().requires_grad_(True)
    wr = conv.weight.detach().double().requires_grad_(True)
    br = conv.bias.detach().double().requires_grad_(True) if bias else None
    yr = F.conv2d(xr, wr, br, padding=1)
    yr.backward(dy.double())
    scale = yr.abs().max().item() + 1
    torch.testing.assert_close(y.double(), yr, rtol=1e-4, atol=2e-5 * scale)
    torch.testing.assert_close(x.grad.double(), xr.grad, rtol=1e-4,
                               atol=2e-5 * (xr.grad.abs().max().item() + 1))
    torch.testing.assert_close(conv.weight.grad.double(), wr.grad, rtol=1e-4,
                               atol=2e-5 * (wr.grad.abs().max().item() + 1))
    if bias:
        torch.testing.assert_close(conv.bias.grad.double(), br.grad, rtol=1e-4, atol=1e-3)


def test_transform_cache_follows_weight_updates():
    conv = WinogradConv2d(8, 16, 3, padding=1, bias=False).to(cuda)
    x = torch.randn(2, 8, 10, 10, device=cuda)
    a = conv(x)
    with torch.no_grad():
        conv.weight.mul_(2)  # in-place update bumps the version -> new transform
    b = conv(x)
    torch.testing.assert_close(b, 2 * a, rtol=1e-5, atol=1e-5)
    clone = copy.deepcopy(conv)
    torch.testing.assert_close(clone(x), b)


def test_same_state_dict_as_conv2d():
    conv = WinogradConv2d(4, 6, 3, padding=1)
    plain = torch.nn.Conv2d(4, 6, 3, padding=1)
    assert conv.state_dict().keys() == plain.state_dict().keys()


def test_functional_falls_back_for_other_configs():
    x = torch.randn(1, 4, 9, 9, device=cuda)
    w = torch.randn(6, 4, 5, 5, device=cuda)
    torch.testing.assert_close(winograd_conv2d(x, w), F.conv2d(x, w, padding=1))


@pytest.mark.parametrize('shape', SHAPES + [(2, 70, 40, 10, 12), (1, 8, 8, 2, 2)])
def test_weight_gradient_kernel(shape):
    n, c, k, h, w = shape
    torch.manual_seed(1)
    x = torch.randn(n, c, h, w, device=cuda)
    dy = torch.randn(n, k, h, w, device=cuda)
    ops = _ext.require(x)
    want = torch.ops.aten.convolution_backward(
        dy.double(), x.double(), torch.zeros(k, c, 3, 3, device=cuda, dtype=torch.float64), None,
        [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]
    for variant in (0, 2):
        for splits in (0, 1, 3):
            got = ops.wino_wgrad(x, dy, splits, variant)
            torch.testing.assert_close(got.double(), want, rtol=1e-4,
                                       atol=2e-5 * (want.abs().max().item() + 1))


def test_direct_ops_small_channels():
    # the module routes C < 8 to MIOpen; the kernel itself must still be right there
    x = torch.randn(2, 5, 9, 7, device=cuda)
    w = torch.randn(70, 5, 3, 3, device=cuda)
    ops = _ext.require(x)
    for variant in (0, 1, 2):
        y = ops.wino_conv(x, ops.wino_weight(w, False), None, 70, variant, 0)
        torch.testing.assert_close(y.double(), _ref(x, w), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('shape', [(2, 64, 64, 24, 24), (1, 24, 130, 14, 10), (3, 16, 96, 9, 12),
                                   (2, 40, 64, 8, 8), (1, 3, 64, 16, 16), (2, 5, 70, 7, 9),
                                   (1, 16, 8, 1, 1), (4, 32, 32, 33, 2), (2, 256, 128, 12, 12),
                                   (1, 64, 192, 20, 36)])
@pytest.mark.parametrize('splits', [0, 1, 3])
@pytest.mark.parametrize('variant', [4, 5, 6, 7, 12, 14, 15, 18])
def test_f4_forward_and_flip(shape, splits, variant):
    # Winograd F(4x4,3x3): edge tiles (H, W not multiples of 4), padded channels, split-K,
    # and backward-data through the flipped weight transform
    n, c, k, h, w = shape
    torch.manual_seed(3)
    x = torch.randn(n, c, h, w, device=cuda)
    wt = torch.randn(k, c, 3, 3, device=cuda) / (3 * c ** 0.5)
    b = torch.randn(k, device=cuda)
    ops = _ext.require(x)
    y = ops.wino4_conv(x, ops.wino4_weight(wt, False), b, k, variant, splits)
    want = _ref(x, wt, b)
    torch.testing.assert_close(y.double(), want, rtol=1e-4,
                               atol=5e-5 * (want.abs().max().item() + 1))
    dy = torch.randn(n, k, h, w, device=cuda)
    dx = ops.wino4_conv(dy, ops.wino4_weight(wt, True), None, c, variant, splits)
    want_dx = torch.ops.aten.convolution_backward(
        dy.double(), x.double(), wt.double(), None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
        [True, False, False])[0]
    torch.testing.assert_close(dx.double(), want_dx, rtol=1e-4,
                               atol=5e-5 * (want_dx.abs().max().item() + 1))


@pytest.mark.parametrize('shape', [(2, 64, 64, 24, 24), (1, 24, 130, 14, 10), (3, 16, 96, 9, 12),
                                   (2, 40, 64, 8, 8), (1, 3, 64, 16, 16), (2, 5, 70, 7, 9),
                                   (1, 16, 8, 1, 1), (4, 32, 32, 33, 2), (2, 256, 128, 12, 12),
                                   (5, 64, 33, 20, 36)])
@pytest.mark.parametrize('splits', [0, 1, 3, 1000])
@pytest.mark.parametrize('variant', [0, 1, 2])
def test_f4_wgrad(shape, splits, variant):
    # F(4x4,3x3) weight gradient: edge tiles, channel blocks past C / K, split tiles
    # (1000 is capped at the step count); variant 2 = the split-bf16 batched GEMM (rows
    # past K, columns past C, 16-tile steps past the last tile)
    n, c, k, h, w = shape
    torch.manual_seed(5)
    x = torch.randn(n, c, h, w, device=cuda)
    dy = torch.randn(n, k, h, w, device=cuda)
    got = _ext.require(x).wino4_wgrad(x, dy, splits, variant)
    want = torch.ops.aten.convolution_backward(
        dy.double(), x.double(), torch.zeros(k, c, 3, 3, device=cuda, dtype=torch.double), None,
        [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]
    torch.testing.assert_close(got.double(), want, rtol=1e-4,
                               atol=5e-5 * (want.abs().max().item() + 1))


@pytest.mark.parametrize('variant', [0, 1, 2])
def test_f4_wgrad_accumulates_into_existing_gradient(variant):
    """``into``: the weight gradient is added to an existing ``.grad`` (gradient-accumulation
    fusion), split partials included."""
    n, c, k, h, w = 3, 70, 130, 13, 13
    torch.manual_seed(6)
    x = torch.randn(n, c, h, w, device=cuda)
    dy = torch.randn(n, k, h, w, device=cuda)
    base = torch.randn(k, c, 3, 3, device=cuda)
    into = base.clone()
    got = _ext.require(x).wino4_wgrad(x, dy, 2, variant, into)
    assert got.data_ptr() == into.data_ptr()
    want = base.double() + torch.ops.aten.convolution_backward(
        dy.double(), x.double(), torch.zeros(k, c, 3, 3, device=cuda, dtype=torch.double), None,
        [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [False, True, False])[1]
    torch.testing.assert_close(got.double(), want, rtol=1e-4,
                               atol=5e-5 * (want.abs().max().item() + 1))


@pytest.mark.parametrize('variant', [0, 1, 2])
@pytest.mark.parametrize('shape', [(2, 64, 64, 24, 24), (1, 24, 130, 14, 10), (3, 16, 96, 9, 12),
                                   (2, 40, 64, 8, 8)])
@pytest.mark.parametrize('splits', [0, 1, 3])
def test_forward_variants_and_splits(variant, shape, splits):
    # variant 2 = double-buffered one-workgroup-per-CU kernel (paired 16-byte stores when
    # W % 4 == 0 and H is even; plain stores otherwise)
    n, c, k, h, w = shape
    torch.manual_seed(2)
    x = torch.randn(n, c, h, w, device=cuda)
    wt = torch.randn(k, c, 3, 3, device=cuda)
    b = torch.randn(k, device=cuda)
    ops = _ext.require(x)
    y = ops.wino_conv(x, ops.wino_weight(wt, False), b, k, variant, splits)
    want = _ref(x, wt, b)
    torch.testing.assert_close(y.double(), want, rtol=1e-4,
                               atol=2e-5 * (want.abs().max().item() + 1))


def test_weight_update_through_data_is_seen_by_the_next_pipeline_step():
    """``p.data.copy_`` does not bump ``_version``; the per-step cache key does."""
    from torchgpipe_amd import GPipe
    from torchgpipe_amd.ops.conv import WinogradConv2d
    torch.manual_seed(0)
    conv = WinogradConv2d(16, 16, 3, padding=1, bias=False).cuda()
    model = GPipe(torch.nn.Sequential(conv), [1], devices=[0], chunks=2)
    x = torch.randn(4, 16, 12, 12, device='cuda')
    with torch.no_grad():
        model(x)  # fills the cache
        conv.weight.data.copy_(torch.randn_like(conv.weight))
        got = model(x)
    want = F.conv2d(x.double(), conv.weight.double(), padding=1)
    assert ((got.double() - want).norm() / want.norm()).item() < 1e-5


def test_cache_budget_zero_keeps_no_transforms(monkeypatch):
    from torchgpipe_amd.ops import conv as convmod
    monkeypatch.delenv('TGPIPE_WINOGRAD_CACHE_MB', raising=False)
    monkeypatch.setitem(convmod._DEVICE_BUDGET, torch.device('cuda', 0), 0)  # hold_cache
    torch.manual_seed(1)
    layer = convmod.WinogradConv2d(16, 16, 3, padding=1, bias=False).cuda()
    x = torch.randn(2, 16, 12, 12, device='cuda', requires_grad=True)
    before = convmod.cache_bytes()
    y = layer(x)
    y.sum().backward()
    assert convmod.cache_bytes() == before
    want = F.conv2d(x.double(), layer.weight.double(), padding=1)
    assert ((y.double() - want).norm() / want.norm()).item() < 1e-5


# -- batched-GEMM F(4x4) (bg_weight / bg_conv): every N-tile width and split-K --------------

BG_SHAPES = [  # (N, C, K, H, W)
    (16, 512, 512, 24, 24),    # 576 tiles: BN 96
    (16, 1024, 1024, 12, 12),  # 144 tiles: BN 48
    (16, 256, 512, 6, 6),      # 64 tiles: BN 64
    (3, 70, 130, 13, 11),      # ragged channels / planes: every padding path
    (1, 16, 8, 5, 7),
    (40, 128, 96, 12, 12),     # 360 tiles: BN 128
    # the split-bf16 input image at 4 channels per thread (the smaller grids above take 2
    # or 1: launch_bg_conv)
    (4, 64, 48, 192, 192),
]


def _bg_run(x, wt, bias, flip, kind, emu, bn=0, splits=0, waves=0, sub=0):
    ops = _ext.require(x)
    out_channels = wt.shape[1] if flip else wt.shape[0]
    return ops.bg_conv(x, ops.bg_weight(wt, flip, kind, emu=emu), bias, out_channels, bn,
                       splits, kind, waves, sub, emu=emu)


@pytest.mark.parametrize('emu', [0, 1], ids=['f32', 'split-bf16'])
@pytest.mark.parametrize('shape', BG_SHAPES)
@pytest.mark.parametrize('flip', [False, True])
@pytest.mark.parametrize('kind', [4, 2])
def test_batched_gemm_winograd_matches_conv2d(shape, flip, kind, emu):
    """Forward (flip=False) and backward-data (flip=True: the rotated, transposed weights)
    of the batched-GEMM path, F(4x4) and F(2x2), f32 and split-bf16 GEMMs, against fp64."""
    n, c, k, h, w = shape
    torch.manual_seed(0)
    wt = torch.randn(k, c, 3, 3, device=cuda) / (3 * c ** 0.5)
    if flip:  # dx = conv_transpose(dy, w): input has k channels, output c
        x = torch.randn(n, k, h, w, device=cuda)
        want = F.conv_transpose2d(x.double(), wt.double(), padding=1)
        got = _bg_run(x, wt, None, True, kind, emu)
    else:
        x = torch.randn(n, c, h, w, device=cuda)
        b = torch.randn(k, device=cuda)
        want = _ref(x, wt, b)
        got = _bg_run(x, wt, b, False, kind, emu)
    torch.testing.assert_close(got.double(), want, rtol=1e-4,
                               atol=2e-5 * (want.abs().max().item() + 1))


@pytest.mark.parametrize('shape', BG_SHAPES[:4])
@pytest.mark.parametrize('kind', [4, 2])
def test_split_bf16_gemm_is_as_accurate_as_f32(shape, kind):
    """The split-bf16 products (six bf16 MFMAs per f32 product) carry no more error against
    fp64 than the f32 MFMA GEMM of the same transformed operands: the Winograd transform
    dominates both, the split adds < 2^-22 per product."""
    n, c, k, h, w = shape
    torch.manual_seed(2)
    wt = torch.randn(k, c, 3, 3, device=cuda) / (3 * c ** 0.5)
    x = torch.randn(n, c, h, w, device=cuda)
    want = _ref(x, wt)
    err = {}
    for emu in (0, 1):
        got = _bg_run(x, wt, None, False, kind, emu).double()
        err[emu] = ((got - want).norm() / want.norm()).item()
    assert err[1] <= 1.25 * err[0] + 1e-7, err


@pytest.mark.parametrize('emu', [0, 1], ids=['f32', 'split-bf16'])
@pytest.mark.parametrize('waves,bn,sub', [(4, 48, 1), (4, 64, 1), (4, 96, 1), (4, 128, 1),
                                          (4, 48, 2), (4, 64, 2), (4, 96, 2), (4, 128, 2),
                                          (8, 64, 1), (8, 96, 1), (8, 128, 1), (8, 144, 1)])
@pytest.mark.parametrize('splits', [1, 3])
def test_batched_gemm_tile_shapes_and_splits(waves, bn, sub, splits, emu):
    """Every tile shape (split-bf16: 4 waves x 64 / 96 / 128, one step per stage; other
    requests fall back to its automatic width) with and without split-K."""
    n, c, k, h, w = 4, 96, 300, 20, 20
    torch.manual_seed(1)
    x = torch.randn(n, c, h, w, device=cuda)
    wt = torch.randn(k, c, 3, 3, device=cuda) / (3 * c ** 0.5)
    got = _bg_run(x, wt, None, False, 4, emu, bn, splits, waves, sub)
    want = _ref(x, wt)
    torch.testing.assert_close(got.double(), want, rtol=1e-4,
                               atol=2e-5 * (want.abs().max().item() + 1))


@pytest.mark.parametrize('kind', ['winograd', 'gemm'])
def test_retain_graph_second_backward_accumulates(kind):
    """A second backward through the same graph (``retain_graph=True``) doubles every
    gradient: the fused ``.grad`` accumulation of the first pass must not break the second
    (it falls back to returning the weight gradient to autograd)."""
    from torchgpipe_amd.ops.convbn import GemmConv2d
    torch.manual_seed(0)
    if kind == 'winograd':
        conv = WinogradConv2d(32, 64, 3, padding=1, bias=False).to(cuda)
        x = torch.randn(2, 32, 24, 24, device=cuda, requires_grad=True)
    else:
        conv = GemmConv2d(64, 8, kernel_size=1, bias=False).to(cuda)
        x = torch.randn(2, 64, 24, 24, device=cuda, requires_grad=True)
    y = conv(x)
    dy = torch.randn_like(y)
    y.backward(dy, retain_graph=True)
    gw1, gx1 = conv.weight.grad.clone(), x.grad.clone()
    y.backward(dy)
    torch.testing.assert_close(conv.weight.grad, 2 * gw1, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(x.grad, 2 * gx1, rtol=1e-5, atol=1e-5)


def test_cache_budget_sizing_modes(monkeypatch):
    """size_cache_budget: half of what the uncached step left free (default), or a
    fraction of its peak (the memory-lean mode), never above 5 % of the device."""
    from torchgpipe_amd.ops import conv as convmod
    dev = torch.device('cuda', 0)
    monkeypatch.setitem(convmod._DEVICE_BUDGET, dev, 0)
    total = torch.cuda.get_device_properties(dev).total_memory
    cap = total // 20
    assert convmod.size_cache_budget(dev, total - (1 << 30), fraction=None) == \
        min(cap, (1 << 30) // 2)
    # the pre-split weights get at most half of what the step and the cache left free
    assert convmod.presplit_budget_mb == min(convmod.PRESPLIT_MB, 256)
    assert convmod.size_cache_budget(dev, 1 << 30, fraction=0.15) == int(0.15 * (1 << 30))
    assert convmod.presplit_budget_mb == 0
    assert convmod.size_cache_budget(dev, total // 2, fraction=None) == cap
    assert convmod.presplit_budget_mb == convmod.PRESPLIT_MB
    convmod._presplit_budget(-1)


def test_module_weight_gradient_picks_split_bf16_gemm_for_deep_layers():
    """``WinogradConv2d``'s weight gradient at 512 channels on >= 320 tiles runs the
    split-bf16 batched GEMM (variant 2) and matches float64."""
    from torchgpipe_amd.ops import conv as conv_mod
    torch.manual_seed(9)
    m = conv_mod.WinogradConv2d(512, 512, 3, padding=1, bias=False).to(cuda)
    x = torch.randn(3, 512, 48, 48, device=cuda, requires_grad=True)
    assert conv_mod._wgrad_f4_variant(x, m.weight) == 2
    y = m(x)
    g = torch.randn_like(y)
    y.backward(g)
    want = torch.ops.aten.convolution_backward(
        g.double(), x.detach().double(), m.weight.detach().double(), None, [1, 1], [1, 1],
        [1, 1], False, [0, 0], 1, [False, True, False])[1]
    torch.testing.assert_close(m.weight.grad.double(), want, rtol=1e-4,
                               atol=5e-5 * (want.abs().max().item() + 1))


@pytest.mark.parametrize('shape,kind', [((22, 256, 256, 14, 14), 4), ((22, 512, 512, 7, 7), 2),
                                        ((3, 70, 130, 13, 11), 4), ((3, 70, 130, 13, 11), 2),
                                        ((9, 256, 64, 28, 28), 4)])
def test_batched_gemm_output_pass_leaves_batchnorm_statistics(shape, kind):
    """``bg_conv(..., stats=)``: the same output as without (same arithmetic), plus per
    (image group, channel) mean / centred M2 partials that merge to the output's batch
    mean and variance (float64 reference)."""
    n, c, k, h, w = shape
    torch.manual_seed(4)
    ops = _ext.require(torch.empty(1, device=cuda))
    x = torch.randn(n, c, h, w, device=cuda)
    wt = torch.randn(k, c, 3, 3, device=cuda) / (3 * c ** 0.5)
    u = ops.bg_weight(wt, False, kind, emu=1)
    ipg = ops.bg_stats_images(n, h, w, kind)
    groups = -(-n // ipg)
    stats = torch.full((2, groups, k), float('nan'), device=cuda)
    y = ops.bg_conv(x, u, None, k, 0, 0, kind, emu=1, stats=stats)
    y_plain = ops.bg_conv(x, u, None, k, 0, 0, kind, emu=1)
    torch.testing.assert_close(y, y_plain, rtol=0, atol=0)
    counts = torch.tensor([min(ipg, n - g * ipg) * h * w for g in range(groups)],
                          dtype=torch.float64, device=cuda)[:, None]
    mean_g, m2_g = stats[0].double(), stats[1].double()
    total = counts.sum()
    mean = (counts * mean_g).sum(0) / total
    m2 = (m2_g + counts * (mean_g - mean) ** 2).sum(0)
    want = y.double()
    torch.testing.assert_close(mean, want.mean((0, 2, 3)), rtol=1e-5,
                               atol=1e-6 * want.abs().max().item())
    torch.testing.assert_close(m2 / total, want.var((0, 2, 3), unbiased=False), rtol=1e-5,
                               atol=1e-7)
