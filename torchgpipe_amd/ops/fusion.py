"""Conv → BatchNorm (→ ReLU) fusion across the layers of a flat ``nn.Sequential``.

The benchmark ResNet-101 (reference ``benchmarks/models/resnet/bottleneck.py:31-79``) is a
flat sequence of 370 layers -- ``conv1, bn1, relu1, conv2, bn2, relu2, conv3, bn3, ...`` --
because GPipe balances and checkpoints by layer.  Keeping that structure (the reference's
balance tables and state-dict keys apply unchanged) while running each Conv-BN-ReLU run as
one native op needs the layers to cooperate:

* :class:`ConvBN2d` (an ``nn.Conv2d``): when :func:`relink` has linked it to the
  :class:`BatchNormAct2d` right after it (and a :class:`ReLU` after that), its forward
  runs the convolution, the BatchNorm and the ReLU:

  - 1x1 stride-1 convolutions: the implicit-GEMM MFMA kernel with the BatchNorm
    statistics in its epilogue, one finalize + normalise (+ ReLU) pass
    (``ops.convbn.relu_conv_bn`` with ``relu_out``); the backward re-derives the ReLU
    mask from the saved convolution output;
  - 3x3 stride-1 convolutions: the Winograd F(4x4) / batched-GEMM kernels
    (``ops.conv``), then the native BatchNorm(+ReLU) pass (:func:`bn_act`) -- from the
    batched-GEMM output pass's statistics partials where it ran (``conv_with_bn_stats``);
  - strided convolutions (the 7x7 stem, the stride-2 3x3 and 1x1 of each stage's first
    block): the fused native op (implicit-GEMM forward, stride-phase backward-data) for the
    geometries where it measured faster (``STRIDED_FUSED``), MIOpen then :func:`bn_act`
    for the others;

  and marks its output as normalised (and rectified) by that BatchNorm;
* :class:`BatchNormAct2d` passes a marked input through; otherwise it runs the native
  BatchNorm (+ the linked ReLU) or ``nn.BatchNorm2d``;
* :class:`ReLU` passes an input the BatchNorm already rectified through.

Links are only made between consecutive layers of one ``nn.Sequential`` -- one pipeline
partition -- so a balance that separates a convolution from its BatchNorm leaves both
running on their own.  ``GPipe`` and ``PipelineStage`` call :func:`relink` on every
partition after splitting (and after DeferredBatchNorm conversion, whose BatchNorms are
not linked).  Outside training mode, on the CPU, or for non-fp32 tensors every layer runs
its plain PyTorch forward.
"""
import os
from typing import Callable, Dict, Optional

import torch
from torch import Tensor, nn
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext, gradacc
from torchgpipe_amd.ops.conv import WinogradConv2d, conv_with_bn_stats, wino_eligible
from torchgpipe_amd.ops.convbn import (GradSink, _bn_ok, fusable, gemm_conv2d,
                                       gemm_conv_eligible, relu_conv_bn)

__all__ = ['ConvBN2d', 'BatchNormAct2d', 'ReLU', 'Linear', 'relink', 'bn_act', 'add_relu',
           'pending_join']

_LINK = '_tgpipe_link'       # ConvBN2d -> (BatchNormAct2d, relu?)
_RELU = '_tgpipe_relu_next'  # BatchNormAct2d -> a linked ReLU follows
_DONE_BN = '_tgpipe_bn_done'    # tensor mark: id() of the BatchNorm already applied
_DONE_RELU = '_tgpipe_relu_done'  # tensor mark: the ReLU after it too
_PENDING = '_tgpipe_pending'  # tensor mark: (conv, bn) left for the residual join to run
_SINK = '_tgpipe_grad_sink'  # tensor mark: a fused reader accepts this tensor's other gradient
# TGPIPE_GRAD_SINK=0: the residual join returns the identity's gradient to autograd (which
# sums it with conv1's) instead of handing it to conv1's backward-data GEMM
GRAD_SINK = os.environ.get('TGPIPE_GRAD_SINK', '1') != '0'
# TGPIPE_BN_GRAD_ACCUM=0: the native BatchNorm's gamma / beta gradients go back to autograd
# (which adds them per micro-batch) instead of into .grad from the kernel
BN_GRAD_ACCUM = os.environ.get('TGPIPE_BN_GRAD_ACCUM', '1') != '0'


class _BNAct(torch.autograd.Function):
    """Training-mode BatchNorm2d (batch statistics, running-stat EMA) + optional ReLU on the
    native kernels (``csrc/batchnorm.hip``): statistics pass, finalize + normalise (+ ReLU)."""

    @staticmethod
    def forward(ctx, x: Tensor, gamma: Optional[Tensor], beta: Optional[Tensor],  # type: ignore[override]
                bn: nn.BatchNorm2d, relu: bool, part: Optional[Tensor] = None,
                part_images: int = 0) -> Tensor:
        track = bn.track_running_stats and bn.running_mean is not None
        # part: x's statistics partials from its producer (ops/conv.py conv_with_bn_stats)
        y, mean, invstd, sums = _ext.require(x).bn_train_forward(
            x, gamma, beta, None, float(bn.eps),
            bn.running_mean if track else None, bn.running_var if track else None,
            bn.num_batches_tracked if track else None,
            float(bn.momentum) if track else 0.0, relu, part, part_images)
        ctx.save_for_backward(x, mean, invstd, sums, gamma, beta)
        ctx.relu = relu
        ctx.params = (bn.weight, bn.bias)
        return y

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        x, mean, invstd, sums, gamma, beta = ctx.saved_tensors
        # the affine gradients accumulate into .grad in the kernel where autograd would add
        # them (ops/gradacc.py): one launch per micro-batch and BatchNorm fewer
        fused = [gradacc.target(p) if ctx.needs_input_grad[k + 1] and BN_GRAD_ACCUM
                 else (False, None) for k, p in enumerate(ctx.params)]
        dx, dgamma, dbeta = _ext.require(dy).bn_train_backward(
            dy.contiguous(), x, mean, invstd, sums, gamma, beta, ctx.relu,
            fused[0][1], fused[1][1])
        grads = [dgamma if ctx.needs_input_grad[1] else None,
                 dbeta if ctx.needs_input_grad[2] else None]
        for k, ((fuse, into), p) in enumerate(zip(fused, ctx.params)):
            if fuse:
                if into is None:
                    gradacc.commit(p, grads[k])
                grads[k] = None
        ctx.params = None
        return (dx, grads[0], grads[1], None, None, None, None)


def _native_bn_ok(bn: nn.BatchNorm2d, x: Tensor) -> bool:
    return _bn_ok(bn, x) and x.numel() > 0 and _ext.available()


def bn_act(x: Tensor, bn: nn.BatchNorm2d, relu: bool, part: Optional[Tensor] = None,
           part_images: int = 0) -> Tensor:
    """``relu(bn(x))`` (or ``bn(x)``) in training mode on the native kernels; callers check
    :func:`_native_bn_ok` first.  ``part``: x's (mean, M2) partials from its producer."""
    return _BNAct.apply(x.contiguous(), bn.weight, bn.bias, bn, relu, part, part_images)


def _mark(y: Tensor, bn: nn.Module, relu: bool) -> Tensor:
    setattr(y, _DONE_BN, id(bn))
    if relu:
        setattr(y, _DONE_RELU, True)
    return y


class _AddReLU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a: Tensor, b: Tensor) -> Tensor:  # type: ignore[override]
        y = _ext.require(a).add_relu_forward(a, b)
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        (y,) = ctx.saved_tensors
        g = torch.ops.aten.threshold_backward(dy, y, 0.0)
        return g, g


def add_relu(a: Tensor, b: Tensor) -> Tensor:
    """``relu(a + b)`` in one pass on the GPU (fp32, same shape); marked for a following
    :class:`ReLU` to pass through."""
    if (a.is_cuda and a.dtype == torch.float32 and b.dtype == torch.float32
            and a.shape == b.shape and a.device == b.device and _ext.available()):
        y = _AddReLU.apply(a, b)
    else:
        y = F.relu(a + b)
    setattr(y, _DONE_RELU, True)
    return y


def pending_join(x: Tensor, join: nn.Module, identity: Tensor) -> Optional[Tensor]:
    """``relu(bn(conv(x)) + identity)`` when ``x`` is the input a linked :class:`ConvBN2d`
    left for the residual join ``join`` (ResNet's ``conv3, bn3, residual, relu3``): one
    implicit-GEMM convolution with the BatchNorm statistics in its epilogue and one
    normalise + add + ReLU pass, so the BatchNorm output never round-trips through memory.
    ``None`` when ``x`` carries no such pending work."""
    pend = getattr(x, _PENDING, None)
    if pend is None or pend[2] is not join:
        return None
    conv, bn, _ = pend
    n, _, h, w = x.shape
    if identity.shape != (n, conv.out_channels, h, w) or identity.dtype != x.dtype:
        y = relu_conv_bn(x, [(conv, 0)], bn, relu=False) + identity
        y = F.relu(y)
    else:
        # identity is the block input that conv1 read: its gradient goes to conv1's
        # backward-data GEMM (GradSink) instead of through autograd's sum
        sink = getattr(identity, _SINK, None)
        if sink is not None and (sink.claimed or not identity.is_contiguous()):
            sink = None
        if sink is not None:
            sink.claimed = True
        y = relu_conv_bn(x, [(conv, 0)], bn, relu=False, add=identity.contiguous(),
                         relu_out=True, sink_out=sink)
    setattr(y, _DONE_RELU, True)
    return y


def relu_follows(module: nn.Module) -> bool:
    """Whether :func:`relink` linked a :class:`ReLU` after ``module`` (a layer that can apply
    it itself, e.g. ResNet's residual join: ``fuses_relu = True``)."""
    return bool(module.__dict__.get(_RELU, False))


def _pointwise(conv: nn.Conv2d) -> bool:
    return (tuple(conv.kernel_size) == (1, 1) and tuple(conv.stride) == (1, 1)
            and tuple(conv.padding) == (0, 0))  # type: ignore[arg-type]


# strided convolutions: geometry -> whether the fused implicit-GEMM op (its backward-data
# on MIOpen where that timed faster) beat MIOpen + the native BatchNorm, forward + backward
_STRIDED: Dict[tuple, bool] = {}
# TGPIPE_STRIDED_CHOICE=1: time both ways on the first eager call of a geometry (the
# offline measurement's method); default: the shipped measured set below
STRIDED_CHOICE = os.environ.get('TGPIPE_STRIDED_CHOICE', '0') != '0'
# Strided Conv-BN(-ReLU) geometries (in channels, out channels, kernel, stride, padding,
# input height) where the fused native op -- implicit-GEMM forward with the BatchNorm
# statistics in its epilogue, stride-phase backward-data -- measured faster than MIOpen +
# the native BatchNorm at ResNet-101's pipeline-1 micro-batch of 110
# (benchmarks/diag/resnet_strided_probe.py, profiles/r4/resnet/resnet_strided_probe_r4ac.jsonl:
# 1386 / 1612 / 1178 vs 1440 / 1714 / 1355 us forward + backward).  Round 6 re-timed every
# strided geometry on the split-bf16 kernels at 15 / 22 / 36 / 110 images
# (benchmarks/diag/strided_picks.py, profiles/r6/strided_picks.json): the 7x7 stem and the
# 28^2 / 14^2 downsamples now win at every size too (ResNet p4 stage 3 / p8 stage 3 kernel
# time -1.1 / -1.4 %, 3.8 k / 1.9 k launches fewer per step: profiles/r6/strided/); the 28^2
# 3x3 wins at 15 and 36 images but not at 22 or 110 and stays on MIOpen.
STRIDED_FUSED = frozenset({
    (3, 64, (7, 7), (2, 2), (3, 3), 224),
    (128, 128, (3, 3), (2, 2), (1, 1), 56),
    (256, 512, (1, 1), (2, 2), (0, 0), 56),
    (512, 1024, (1, 1), (2, 2), (0, 0), 28),
    (512, 512, (3, 3), (2, 2), (1, 1), 14),
    (1024, 2048, (1, 1), (2, 2), (0, 0), 14),
})


def _strided_fused(conv: nn.Conv2d, bn: nn.BatchNorm2d, x: Tensor, relu: bool) -> bool:
    """Whether one strided Conv-BN(-ReLU) runs as the fused native op: the shipped measured
    set (``STRIDED_FUSED``), or with ``TGPIPE_STRIDED_CHOICE=1`` both ways timed on the first
    eager call of its geometry (on copies of the layers: the real ones' parameters,
    gradients and running statistics are untouched; inside a stream capture an undecided
    geometry stays on MIOpen)."""
    if not STRIDED_CHOICE:
        return (conv.in_channels, conv.out_channels, tuple(conv.kernel_size), tuple(conv.stride),
                tuple(conv.padding), x.shape[2]) in STRIDED_FUSED  # type: ignore[arg-type]
    key = (tuple(x.shape), conv.out_channels, tuple(conv.kernel_size), tuple(conv.stride),
           tuple(conv.padding), relu, x.device)  # type: ignore[arg-type]
    hit = _STRIDED.get(key)
    if hit is not None:
        return hit
    if torch.cuda.is_current_stream_capturing():
        return False
    import copy
    c2, b2 = copy.deepcopy(conv), copy.deepcopy(bn)
    for m in (c2, b2):
        m.__dict__.pop(_LINK, None)
        m.__dict__.pop('_wt_cache', None)
    xg = x.detach().clone().requires_grad_(x.requires_grad)

    def library() -> Tensor:
        return bn_act(F.conv2d(xg, c2.weight, None, c2.stride, c2.padding), b2, relu)

    def fused() -> Tensor:
        return relu_conv_bn(xg, [(c2, 0)], b2, relu=False, relu_out=relu)

    with torch.enable_grad():
        dy = torch.randn_like(library())

        def timed(fn: Callable[[], Tensor]) -> float:
            best = float('inf')
            for rep in range(3):  # first: warm-up (plans, MIOpen's find step)
                a = torch.cuda.Event(enable_timing=True)
                b = torch.cuda.Event(enable_timing=True)
                a.record()
                fn().backward(dy)
                b.record()
                b.synchronize()
                if rep:
                    best = min(best, a.elapsed_time(b))
            return best

        lib_ms, fused_ms = timed(library), timed(fused)
    pick = fused_ms < 0.97 * lib_ms
    _STRIDED[key] = pick
    return pick


class ConvBN2d(WinogradConv2d):
    """``nn.Conv2d`` (same parameters) that runs its linked BatchNorm (and ReLU) with it."""

    def forward(self, input: Tensor) -> Tensor:
        link = self.__dict__.get(_LINK)
        wino = self.padding_mode == 'zeros' and wino_eligible(
            input, self.weight, self.stride, self.padding, self.dilation, self.groups)
        if link is not None and self.padding_mode == 'zeros':
            bn, relu, join = link
            if (join is not None and self.bias is None and _pointwise(self)
                    and _native_bn_ok(bn, input) and fusable(input, [self], bn)):
                # the residual join right after the BatchNorm runs this convolution, the
                # BatchNorm, the identity add and the ReLU as one op (pending_join)
                out = input.view_as(input)
                setattr(out, _PENDING, (self, bn, join))
                setattr(out, _DONE_BN, id(bn))
                return out
            if self.bias is None and _native_bn_ok(bn, input):
                if wino:
                    # the batched-GEMM Winograd's output pass leaves the BatchNorm partials
                    with_stats = conv_with_bn_stats(self, input)
                    if with_stats is not None:
                        z, part, images = with_stats
                        return _mark(bn_act(z, bn, relu, part, images), bn, relu)
                    z = WinogradConv2d.forward(self, input)
                    return _mark(bn_act(z, bn, relu), bn, relu)
                if _pointwise(self) and fusable(input, [self], bn):
                    sink = None
                    if GRAD_SINK and relu and input.requires_grad and input.is_contiguous():
                        # (a residual join reading the same tensor may hand its gradient
                        # over: accumulated by this op's backward-data GEMM)
                        sink = GradSink()
                        setattr(input, _SINK, sink)
                    y = relu_conv_bn(input, [(self, 0)], bn, relu=False, relu_out=relu,
                                     sink_in=sink)
                    return _mark(y, bn, relu)
                if fusable(input, [self], bn) and _strided_fused(self, bn, input, relu):
                    y = relu_conv_bn(input, [(self, 0)], bn, relu=False, relu_out=relu)
                    return _mark(y, bn, relu)
                z = gradacc.library_conv2d(input, self)  # strided: MIOpen
                return _mark(bn_act(z, bn, relu), bn, relu)
        if wino:
            return WinogradConv2d.forward(self, input)
        if _pointwise(self) and gemm_conv_eligible(input, self):
            return gemm_conv2d(input, self)
        return gradacc.library_conv2d(input, self)


class Linear(nn.Linear):
    """``nn.Linear`` (same parameters) whose gradients are accumulated into ``.grad`` by its
    own backward (``ops/gradacc.py`` ``linear``): no ``AccumulateGrad`` node shared by
    micro-batches of different lanes."""

    def forward(self, input: Tensor) -> Tensor:
        return gradacc.linear(input, self)


class BatchNormAct2d(nn.BatchNorm2d):
    """``nn.BatchNorm2d`` (same parameters and buffers) that a linked :class:`ConvBN2d` may
    have applied already, and that runs natively with a linked :class:`ReLU` fused."""

    def forward(self, input: Tensor) -> Tensor:
        if getattr(input, _DONE_BN, None) == id(self):
            return input
        relu = bool(self.__dict__.get(_RELU, False))
        if input.dim() == 4 and _native_bn_ok(self, input):
            y = bn_act(input, self, relu)
            if relu:
                setattr(y, _DONE_RELU, True)
            return y
        return super().forward(input)


class ReLU(nn.ReLU):
    """``nn.ReLU`` that passes through an input its linked BatchNorm already rectified."""

    def forward(self, input: Tensor) -> Tensor:
        if getattr(input, _DONE_RELU, False):
            return input
        return F.relu(input, inplace=self.inplace)


def relink(module: nn.Module) -> int:
    """(Re)link every ``ConvBN2d, BatchNormAct2d[, ReLU]`` run of consecutive children of
    each ``nn.Sequential`` in ``module``; earlier links inside ``module`` are dropped first.
    Returns the number of convolutions linked."""
    for m in module.modules():
        m.__dict__.pop(_LINK, None)
        m.__dict__.pop(_RELU, None)
    linked = 0
    for seq in module.modules():
        if not isinstance(seq, nn.Sequential):
            continue
        kids = list(seq.children())
        for i, m in enumerate(kids):
            inner = getattr(m, 'module', m)  # (a @skippable layer wraps the real module)
            if (type(m) is BatchNormAct2d or getattr(inner, 'fuses_relu', False)) and \
                    i + 1 < len(kids) and type(kids[i + 1]) is ReLU:
                inner.__dict__[_RELU] = True
            if not isinstance(m, ConvBN2d) or i + 1 >= len(kids) or \
                    type(kids[i + 1]) is not BatchNormAct2d:
                continue
            relu = i + 2 < len(kids) and type(kids[i + 2]) is ReLU
            join = None
            if not relu and i + 3 < len(kids) and type(kids[i + 3]) is ReLU:
                inner = getattr(kids[i + 2], 'module', kids[i + 2])
                if getattr(inner, 'fuses_residual_bn', False):
                    join = inner  # conv, bn, residual join, relu: see pending_join
            m.__dict__[_LINK] = (kids[i + 1], relu, join)
            linked += 1
    return linked
