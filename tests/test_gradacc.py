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
