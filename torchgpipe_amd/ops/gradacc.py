"""Gradient-accumulation fusion: native backward kernels add straight into ``param.grad``.

A GPipe step runs the backward of every layer once per micro-batch, so autograd's
``AccumulateGrad`` launches ``grad += new`` for every parameter of the model
``chunks - 1`` times per step (AmoebaNet-D(18,256) at 32 micro-batches: 831 parameters,
~26 k tiny add kernels, 7 % of the step).  The fused ops of this package
(:mod:`~torchgpipe_amd.ops.convbn` ReLU-Conv-BN and implicit-GEMM convolutions) instead
accumulate the weight gradient in the epilogue of their weight-gradient GEMM and the
BatchNorm affine gradients in their ``dz`` pass, write ``param.grad`` themselves, and
return no gradient to autograd for those parameters (the technique is known as
gradient-accumulation fusion).

It only applies when the result is indistinguishable from autograd's:

* the engine is running ``.backward()`` and will accumulate into this parameter
  (``torch.autograd.grad`` and ``backward(inputs=...)`` that exclude it fall back);
* no ``create_graph`` (grad mode is off inside the backward);
* the parameter has no tensor / post-accumulate hooks;
* an existing ``.grad`` is a plain contiguous fp32 tensor on the same device.

``TGPIPE_FUSED_GRAD_ACCUM=0`` turns it off (plain autograd accumulation).

The parameter's ``AccumulateGrad`` node is looked up once per step and pinned on the
parameter until :func:`release` (called when the next pipeline step starts,
``ops.conv.new_step``).  Pinning it longer would hand the next step's forward the old
node, which PyTorch bound to the stream it was created on: under forward / recompute
lanes that node's stream differs from the producer's, and the engine then warns ("The
AccumulateGrad node's stream does not match ...") and inserts cross-stream syncs.
"""
import os
from typing import Dict, Optional, Tuple
import weakref

import torch
from torch import Tensor

__all__ = ['target', 'commit', 'enabled', 'release']

_ENABLED = os.environ.get('TGPIPE_FUSED_GRAD_ACCUM', '1') != '0'
_ATTR = '_tgpipe_grad_accumulator'
# id(param) -> weak reference (tensors compare elementwise, so no WeakSet)
_PINNED: Dict[int, 'weakref.ref[Tensor]'] = {}


def enabled() -> bool:
    return _ENABLED


def _accumulator(param: Tensor) -> Optional[object]:
    node = getattr(param, _ATTR, None)
    if node is None:
        with torch.enable_grad():
            fn = param.view_as(param).grad_fn
        if fn is None or not fn.next_functions:
            return None
        node = fn.next_functions[0][0]
        # the tensor only holds its AccumulateGrad weakly; keep it for the rest of the step
        setattr(param, _ATTR, node)
        _PINNED[id(param)] = weakref.ref(param)
    return node


def release() -> None:
    """Drop every pinned ``AccumulateGrad`` node (start of a new step)."""
    for ref in _PINNED.values():
        param = ref()
        if param is not None and hasattr(param, _ATTR):
            delattr(param, _ATTR)
    _PINNED.clear()


def target(param: Optional[Tensor]) -> Tuple[bool, Optional[Tensor]]:
    """``(fuse, into)``: whether the caller writes ``param``'s gradient itself, and the
    existing ``.grad`` to accumulate into (``None``: store a fresh gradient via
    :func:`commit`)."""
    if (not _ENABLED or param is None or not param.requires_grad or not param.is_leaf
            or torch.is_grad_enabled() or param._backward_hooks
            or getattr(param, '_post_accumulate_grad_hooks', None)):
        return False, None
    node = _accumulator(param)
    if node is None:
        return False, None
    try:
        if not torch._C._will_engine_execute_node(node):
            return False, None
    except RuntimeError:  # autograd.grad() naming this leaf: let autograd capture it
        return False, None
    grad = param.grad
    if grad is None:
        return True, None
    if (grad.shape != param.shape or grad.dtype != torch.float32 or grad.device != param.device
            or not grad.is_contiguous() or grad.requires_grad or grad.is_sparse):
        return False, None
    return True, grad


def commit(param: Tensor, grad: Tensor) -> None:
    """Store the first micro-batch's gradient (``param.grad`` was ``None``)."""
    if param.grad is None:
        param.grad = grad
    else:  # pragma: no cover - another op accumulated in between
        param.grad.add_(grad)
