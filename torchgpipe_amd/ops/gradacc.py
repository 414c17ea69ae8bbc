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

Deferred weight gradients (:func:`deferred_wgrad`, used by ``PipelineStage.backward``):
an implicit-GEMM weight gradient whose plan splits the reduction over workgroups (most of
AmoebaNet's: few output tiles, a long images x pixels reduction) would reduce its split
partials in a second launch every micro-batch.  Inside the scope each such parameter
instead owns a *slab* of ``splits`` weight-sized slices that persists across the step's
micro-batches: split ``s`` of every micro-batch adds its partial into slice ``s``
(the first one stores), and one flush at the end of the scope sums the slices into
``.grad`` for all parameters at once (a few launches per step instead of one reduction per
parameter and micro-batch; ~9 k launches per AmoebaNet-D(18, 256) step).  The slices are
summed in a fixed order, so the result is bitwise reproducible.  Slabs stay allocated
(``TGPIPE_DEFERRED_WGRAD=0`` turns the deferral off).

The parameter's ``AccumulateGrad`` node is looked up once per step and pinned on the
parameter until :func:`release` (called when the next pipeline step starts,
``ops.conv.new_step``).  Pinning it longer would hand the next step's forward the old
node, which PyTorch bound to the stream it was created on: under forward / recompute
lanes that node's stream differs from the producer's, and the engine then warns ("The
AccumulateGrad node's stream does not match ...") and inserts cross-stream syncs.
"""
import contextlib
import os
from typing import Dict, Iterator, List, Optional, Tuple
import weakref

import torch
from torch import Tensor

__all__ = ['target', 'commit', 'enabled', 'release', 'deferred_wgrad', 'slab', 'deferred',
           'flush_pending', 'pending_snapshot', 'register_pending', 'library_conv2d',
           'linear']

_ENABLED = os.environ.get('TGPIPE_FUSED_GRAD_ACCUM', '1') != '0'
_DEFER_ENABLED = os.environ.get('TGPIPE_DEFERRED_WGRAD', '1') != '0'
_SLAB_ATTR = '_tgpipe_wgrad_slab'
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


# -- deferred weight gradients -------------------------------------------------------------

class _Deferral:
    """Per-device state of :func:`deferred_wgrad`: scope depth, step number, and the slabs
    written in this step (``id(param)`` -> (weak parameter, slab))."""

    __slots__ = ('depth', 'step', 'pending')

    def __init__(self) -> None:
        self.depth = 0
        self.step = 0
        self.pending: Dict[int, Tuple['weakref.ref[Tensor]', Tensor]] = {}


_DEFER: Dict[torch.device, _Deferral] = {}


def _device_key(device: torch.device) -> torch.device:
    device = torch.device(device)
    if device.type == 'cuda' and device.index is None:
        device = torch.device('cuda', torch.cuda.current_device())
    return device


@contextlib.contextmanager
def deferred_wgrad(device: torch.device, enabled: bool = True) -> Iterator[None]:
    """Defer the split weight-gradient reductions of fused ops on ``device`` to the end of
    this scope (one step's backward of every micro-batch).

    On exit the calling thread's current stream on ``device`` sums every touched slab into
    its parameter's ``.grad`` (accumulating into an existing gradient), so everything that
    wrote a slab must be ordered before that stream by then -- as for the fused ops'
    direct ``.grad`` writes.  Nested scopes flush at the outermost exit; a scope left by an
    exception drops the pending partial sums (the step's gradients are incomplete anyway).
    """
    if not enabled or not _ENABLED or not _DEFER_ENABLED:
        yield
        return
    device = _device_key(device)
    if device.type != 'cuda':
        yield
        return
    state = _DEFER.setdefault(device, _Deferral())
    state.depth += 1
    if state.depth == 1:
        state.step += 1
    ok = False
    try:
        yield
        ok = True
    finally:
        state.depth -= 1
        if state.depth == 0:
            if ok:
                flush_pending(device)
            else:
                state.pending.clear()


def slab(param: Tensor) -> Tuple[Optional[Tensor], bool]:
    """``(slab, first)`` for a fused weight-gradient kernel about to write ``param``'s
    gradient: the parameter's persistent slab (``None`` outside a deferral scope) and
    whether this is the step's first write into it (store rather than add)."""
    state = _DEFER.get(param.device)
    if state is None or state.depth == 0:
        return None, False
    entry: Optional[List] = getattr(param, _SLAB_ATTR, None)
    if entry is None or entry[0].device != param.device:
        entry = [torch.empty(0, device=param.device, dtype=torch.float32), -1]
        setattr(param, _SLAB_ATTR, entry)
    return entry[0], entry[1] != state.step


def deferred(param: Tensor, slab: Tensor, result: Optional[Tensor]) -> bool:
    """Whether the kernel deferred ``param``'s gradient into ``slab`` (it returned the slab
    itself); if so, mark the slab as written in this step and pending its flush."""
    if result is None or slab is None or slab.numel() == 0 or \
            result.data_ptr() != slab.data_ptr():
        return False
    state = _DEFER[param.device]
    entry = getattr(param, _SLAB_ATTR)
    entry[1] = state.step
    state.pending[id(param)] = (weakref.ref(param), slab)
    return True


def flush_pending(device: torch.device) -> None:
    """Sum the slabs written in this step into ``.grad`` (one launch per 24 parameters)."""
    device = _device_key(device)
    state = _DEFER.get(device)
    if state is None or not state.pending:
        return
    items = list(state.pending.values())
    state.pending.clear()
    slabs: List[Tensor] = []
    grads: List[Tensor] = []
    accumulate: List[int] = []
    for ref, sb in items:
        param = ref()
        if param is None:
            continue
        grad = param.grad
        if grad is None:
            grad = torch.empty_like(param, memory_format=torch.contiguous_format)
            param.grad = grad
            accumulate.append(0)
        else:
            accumulate.append(1)
        slabs.append(sb)
        grads.append(grad)
    if slabs:
        from torchgpipe_amd.ops import _ext
        _ext.require(grads[0]).wgrad_slab_flush(slabs, grads, accumulate)


def pending_snapshot(device: torch.device) -> List[Tuple['weakref.ref[Tensor]', Tensor]]:
    """The slabs written so far in the current deferral scope on ``device`` (before its
    flush).  Captured cell graphs (``parallel/segments.py``) write these slabs again on
    every replay without running the Python that registers them; the pipeline re-registers
    this snapshot in each replayed step (:func:`register_pending`)."""
    state = _DEFER.get(_device_key(device))
    return list(state.pending.values()) if state is not None else []


def register_pending(device: torch.device,
                     items: List[Tuple['weakref.ref[Tensor]', Tensor]]) -> None:
    """Mark ``items`` (from :func:`pending_snapshot`) as written in the current scope, so the
    scope's flush sums them into ``.grad``."""
    state = _DEFER.get(_device_key(device))
    if state is None or state.depth == 0:
        return
    for ref, sb in items:
        param = ref()
        if param is None:
            continue
        entry = getattr(param, _SLAB_ATTR, None)
        if entry is not None:
            entry[1] = state.step
        state.pending.setdefault(id(param), (ref, sb))


# -- library layers with the accumulation fused ----------------------------------------------

def _settle(param: Optional[Tensor], grad: Optional[Tensor], fuse: bool,
            into: Optional[Tensor]) -> Optional[Tensor]:
    """Hand a library-computed gradient to ``.grad`` (fused) or back to autograd."""
    if not fuse or grad is None:
        return grad
    assert param is not None
    if into is None:
        commit(param, grad)
    else:
        into.add_(grad)
    return None


class _LibraryConv(torch.autograd.Function):
    """``F.conv2d`` (MIOpen) whose weight / bias gradients are added into ``.grad`` by the
    backward itself (:func:`target`).  Under forward / recompute lanes the micro-batches of
    one step back-propagate on different streams; a parameter left to autograd has one
    ``AccumulateGrad`` node shared by all of them, bound to one stream, and its gradients
    came out wrong across micro-batches under PyTorch 2.10 (``tests/test_overlap_recompute.py``
    ResNet case; ``profiles/KERNELS.md``).  Here the add runs on the backward's own stream,
    which the engine orders micro-batch after micro-batch."""

    @staticmethod
    def forward(ctx, x: Tensor, weight: Tensor, bias: Optional[Tensor],  # type: ignore[override]
                stride: Tuple[int, ...], padding: Tuple[int, ...], dilation: Tuple[int, ...],
                groups: int) -> Tensor:
        ctx.save_for_backward(x, weight)
        ctx.conf = (list(stride), list(padding), list(dilation), groups)
        ctx.params = (weight, bias)
        return torch.nn.functional.conv2d(x, weight, bias, stride, padding, dilation, groups)

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        x, weight = ctx.saved_tensors
        stride, padding, dilation, groups = ctx.conf
        wparam, bparam = ctx.params
        ctx.params = (None, None)  # a repeated backward (retain_graph) returns them instead
        need = ctx.needs_input_grad
        has_bias = need[2]
        fw = target(wparam) if need[1] else (False, None)
        fb = target(bparam) if has_bias else (False, None)
        dx, dw, db = torch.ops.aten.convolution_backward(
            dy, x, weight, [weight.shape[0]] if has_bias else None, stride, padding, dilation,
            False, [0, 0], groups, [need[0], need[1], has_bias])
        dw = _settle(wparam, dw if need[1] else None, *fw)
        db = _settle(bparam, db if has_bias else None, *fb)
        return dx if need[0] else None, dw, db, None, None, None, None


def library_conv2d(x: Tensor, conv: torch.nn.Conv2d) -> Tensor:
    """``conv(x)`` on the library convolution with the gradient accumulation fused (GPU,
    zero padding); ``conv.forward`` otherwise."""
    if not (_ENABLED and x.is_cuda and conv.padding_mode == 'zeros'
            and isinstance(conv.padding, tuple)):
        return torch.nn.Conv2d.forward(conv, x)
    return _LibraryConv.apply(x, conv.weight, conv.bias, conv.stride, conv.padding,
                              conv.dilation, conv.groups)


class _Linear(torch.autograd.Function):
    """``F.linear`` whose weight / bias gradients are accumulated by the backward: the
    weight's as one GEMM with beta = 1 straight into ``.grad`` (``addmm_``), no separate
    add.  See :class:`_LibraryConv` for why."""

    @staticmethod
    def forward(ctx, x: Tensor, weight: Tensor,  # type: ignore[override]
                bias: Optional[Tensor]) -> Tensor:
        ctx.save_for_backward(x, weight)
        ctx.params = (weight, bias)
        return torch.nn.functional.linear(x, weight, bias)

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        x, weight = ctx.saved_tensors
        wparam, bparam = ctx.params
        ctx.params = (None, None)
        need = ctx.needs_input_grad
        dy2 = dy.reshape(-1, dy.shape[-1])
        x2 = x.reshape(-1, x.shape[-1])
        dx = dy.matmul(weight) if need[0] else None
        dw = db = None
        if need[1]:
            fuse, into = target(wparam)
            if fuse and into is not None:
                into.addmm_(dy2.t(), x2)
            else:
                dw = _settle(wparam, dy2.t().mm(x2), fuse, into)
        if need[2]:
            db = _settle(bparam, dy2.sum(0), *target(bparam))
        return dx, dw, db


def linear(x: Tensor, layer: torch.nn.Linear) -> Tensor:
    """``layer(x)`` with the gradient accumulation fused (GPU); ``layer.forward`` otherwise."""
    if not (_ENABLED and x.is_cuda):
        return torch.nn.Linear.forward(layer, x)
    return _Linear.apply(x, layer.weight, layer.bias)
