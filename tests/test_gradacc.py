"""Gradient-accumulation fusion policy (ops/gradacc.py) with a CPU stand-in op."""
import torch
from torch import nn

from torchgpipe_amd.ops import gradacc


class _Scale(torch.autograd.Function):
    """y = x * w; the backward writes w's gradient itself when gradacc allows it."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x)
        ctx.w = w
        return x * w

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        dw = (g * x).sum(0)
        fuse, into = gradacc.target(ctx.w)
        if fuse:
            if into is None:
                gradacc.commit(ctx.w, dw)
            else:
                into.add_(dw)
            dw = None
        return g * ctx.w, dw


def _data():
    torch.manual_seed(0)
    return torch.randn(4, 3, requires_grad=True), nn.Parameter(torch.randn(3))


def test_backward_accumulates_like_autograd():
    x, w = _data()
    for _ in range(3):
        _Scale.apply(x, w).pow(2).sum().backward()
    x2, w2 = _data()
    for _ in range(3):
        (x2 * w2).pow(2).sum().backward()
    torch.testing.assert_close(w.grad, w2.grad)
    torch.testing.assert_close(x.grad, x2.grad)


def test_autograd_grad_falls_back():
    x, w = _data()
    (gw,) = torch.autograd.grad(_Scale.apply(x, w).sum(), [w])
    torch.testing.assert_close(gw, x.detach().sum(0))
    assert w.grad is None
    (gx,) = torch.autograd.grad(_Scale.apply(x, w).sum(), [x])
    assert w.grad is None and gx.shape == x.shape


def test_backward_inputs_excluding_param_leaves_grad_untouched():
    x, w = _data()
    _Scale.apply(x, w).sum().backward(inputs=[x])
    assert w.grad is None and x.grad is not None


def test_hooks_and_create_graph_fall_back():
    x, w = _data()
    seen = []
    w.register_hook(lambda g: seen.append(g))
    _Scale.apply(x, w).sum().backward()
    assert len(seen) == 1 and w.grad is not None
    x, w = _data()
    _Scale.apply(x, w).sum().backward(create_graph=True)
    assert w.grad.grad_fn is not None  # autograd's differentiable accumulation
    w.grad = None  # break the create_graph reference cycle


def test_disabled_switch(monkeypatch):
    monkeypatch.setattr(gradacc, '_ENABLED', False)
    x, w = _data()
    assert gradacc.target(w) == (False, None)
    _Scale.apply(x, w).sum().backward()
    torch.testing.assert_close(w.grad, x.detach().sum(0))


def test_release_drops_pinned_nodes():
    """new_step() unpins the previous step's AccumulateGrad nodes (stream binding)."""
    from torchgpipe_amd.ops.conv import new_step
    x, w = _data()
    _Scale.apply(x, w).sum().backward()
    assert getattr(w, gradacc._ATTR, None) is not None
    new_step()
    assert getattr(w, gradacc._ATTR, None) is None and not gradacc._PINNED
    _Scale.apply(x, w).sum().backward()  # re-acquired on the next backward
    torch.testing.assert_close(w.grad, 2 * x.detach().sum(0))


import pytest  # noqa: E402


@pytest.mark.gpu
@pytest.mark.parametrize('shape', [
    (2, 64, 64, 16), (3, 32, 48, 20),        # F(4x4) fused, one split
    (8, 64, 64, 32),                          # F(4x4) fused, split-K reduction
    (2, 512, 512, 12), (2, 512, 512, 6),      # F(4x4) non-fused
    (2, 64, 96, 6), (32, 64, 96, 6),          # F(2x2), without / with split-K
])
def test_winograd_weight_gradient_accumulates_in_kernel(shape):
    """WinogradConv2d applied to three inputs (three backward calls into one .grad, the
    GPipe micro-batch pattern): the F(4x4) / F(2x2) weight-gradient kernels add into the
    existing .grad themselves; the result matches fp64 PyTorch, and the AccumulateGrad
    node never runs (no autograd accumulation)."""
    from torchgpipe_amd.ops.conv import WinogradConv2d
    n, c, k, hw = shape
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    conv = WinogradConv2d(c, k, 3, padding=1, bias=False).to(dev)
    ref = nn.Conv2d(c, k, 3, padding=1, bias=False).to(dev).double()
    ref.weight.data.copy_(conv.weight.data)
    xs = [torch.randn(n, c, hw, hw, device=dev) for _ in range(3)]
    for x in xs:
        conv(x).square().mean().backward()
        ref(x.double()).square().mean().backward()
    torch.cuda.synchronize()
    err = (conv.weight.grad.double() - ref.weight.grad).norm() / ref.weight.grad.norm()
    assert err < 1e-5, err.item()
