"""Fused ReLU → Conv → BatchNorm for AmoebaNet-D cells on the CDNA4 matrix cores.

Every convolution of AmoebaNet-D (reference ``benchmarks/models/amoebanet/
operations.py:9-114``) is preceded by a ReLU and followed by a BatchNorm, and
except for the stem and the stride-2 3×3 of the reduction cells they are 1×1,
1×7 or 7×1.  :func:`relu_conv_bn` runs such a triplet as one native op
(``csrc/conv_gemm.hip``, ``csrc/batchnorm.hip``, ``csrc/convbn.cpp``):

* forward: an implicit-GEMM ``v_mfma_f32_32x32x2_f32`` kernel reads ``relu(x)``
  straight from the input (no ReLU output tensor), writes the convolution output
  ``z`` and, from its epilogue, per-block (mean, M2) BatchNorm partials; a
  finalize kernel merges them (Chan, fp64), updates the running statistics and
  ``num_batches_tracked``; one elementwise pass normalises and may add the other
  branch of the AmoebaNet node (``left + right``);
* backward: BatchNorm reduction + ``dz`` pass, then the backward-data GEMM with
  the ReLU mask in its epilogue and the split-K weight-gradient GEMM.

:class:`ReLUConvBN` / :class:`FusedChain` are ``nn.Sequential`` subclasses with
the reference's children (``ReLU``, ``Conv2d``, ``BatchNorm2d`` …), so the
state-dict keys are unchanged; they fall back to the eager modules on CPU, in
eval mode, for non-fp32 tensors or unsupported convolutions.
"""
import contextlib
import os
from typing import Dict, Iterator, List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext, gradacc
from torchgpipe_amd.ops.conv import _TransformCache

__all__ = ['relu_conv_bn', 'ReLUConvBN', 'FusedChain', 'conv_supported', 'fused_triplets',
           'fusable', 'disabled', 'GemmConv2d', 'gemm_conv2d', 'gemm_conv_eligible',
           'group_relu_conv_bn', 'groupable']

# TGPIPE_FUSED_CONVBN=0 runs the eager ReLU / Conv2d / BatchNorm2d modules instead.
_ENABLED = os.environ.get('TGPIPE_FUSED_CONVBN', '1') != '0'


@contextlib.contextmanager
def disabled() -> Iterator[None]:
    """Run the eager modules inside this block (numerics oracle, A/B timing)."""
    global _ENABLED
    prev, _ENABLED = _ENABLED, False
    try:
        yield
    finally:
        _ENABLED = prev


Geo = Tuple[int, int, int, int, int, int, int, int]  # kh, kw, sh, sw, ph, pw, oh, ow


def conv_supported(conv: nn.Conv2d) -> bool:
    """Any kernel and stride; no bias, no groups / dilation, zero padding."""
    return (conv.bias is None and conv.groups == 1
            and tuple(conv.dilation) == (1, 1) and conv.padding_mode == 'zeros'
            and isinstance(conv.padding, tuple))


def _geo(conv: nn.Conv2d, offset: int = 0) -> List[int]:
    kh, kw = conv.kernel_size
    sh, sw = conv.stride
    ph, pw = conv.padding  # type: ignore[misc]
    return [kh, kw, sh, sw, ph, pw, offset, offset]


def _bn_ok(bn: nn.Module, x: Tensor) -> bool:
    return (isinstance(bn, nn.BatchNorm2d) and bn.training and x.is_cuda
            and x.dtype == torch.float32 and x.dim() == 4
            and (bn.momentum is not None or not bn.track_running_stats))


# devices whose backward currently runs weight gradients on a side stream -> scope depth
_WGRAD: Dict[torch.device, int] = {}
_WGRAD_STREAMS: Dict[torch.device, torch.cuda.Stream] = {}


@contextlib.contextmanager
def wgrad_stream_scope(device: torch.device, enabled: bool = True) -> Iterator[None]:
    """While active for ``device`` (read on autograd's device threads, so keyed by device
    rather than by thread), fused ops on that device whose weight gradients are
    accumulated by the kernels themselves (``ops/gradacc.py``) run the weight-gradient
    GEMMs on a per-device side stream, concurrently with the backward chain (BatchNorm
    backward, backward-data) that continues on the op's stream.  Pipelines on other
    devices of the process are unaffected.  On exit the caller's current stream on
    ``device`` waits for that side stream, so the gradients are ready for the optimizer.
    Not used inside hipGraph captures.
    """
    device = torch.device(device)
    if device.type == 'cuda' and device.index is None:
        device = torch.device('cuda', torch.cuda.current_device())
    if not enabled:
        yield
        return
    _WGRAD[device] = _WGRAD.get(device, 0) + 1
    try:
        yield
    finally:
        _WGRAD[device] -= 1
        if not _WGRAD[device]:
            del _WGRAD[device]
        stream = _WGRAD_STREAMS.get(device)
        if stream is not None:
            torch.cuda.current_stream(device).wait_stream(stream)


def join_wgrad_stream(device: torch.device) -> None:
    """Order the current stream on ``device`` after the weight-gradient side stream of an
    active :func:`wgrad_stream_scope` (before gradients written there are read: the
    deferred split-gradient flush at the end of a pipeline stage's backward)."""
    stream = _WGRAD_STREAMS.get(device)
    if stream is not None and device in _WGRAD:
        torch.cuda.current_stream(device).wait_stream(stream)


def _wgrad_stream(device: torch.device) -> Optional[torch.cuda.Stream]:
    if device not in _WGRAD or device.type != 'cuda' or torch.cuda.is_current_stream_capturing():
        return None
    stream = _WGRAD_STREAMS.get(device)
    if stream is None:
        stream = _WGRAD_STREAMS[device] = torch.cuda.Stream(device)
    return stream


class GradSink:
    """A gradient handed from one fused op's backward to another's, outside autograd: ResNet's
    residual join deposits the identity's gradient, the block's first convolution (which
    reads the same tensor) accumulates it into its backward-data GEMM -- one pass instead of
    autograd's separate sum of the two gradients (ops/fusion.py pending_join)."""

    __slots__ = ('grad', 'claimed')

    def __init__(self) -> None:
        self.grad: Optional[Tensor] = None
        self.claimed = False


class _ConvBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, add: Optional[Tensor], gamma: Optional[Tensor],  # type: ignore[override]
                beta: Optional[Tensor], bn: nn.BatchNorm2d, geo: List[int], relu: bool,
                relu_out: bool, caches: List[_TransformCache], sinks: Tuple[Optional[GradSink],
                                                                            Optional[GradSink]],
                *weights: Tensor) -> Tensor:
        ops = _ext.require(x)
        track = bn.track_running_stats and bn.running_mean is not None
        y, z, mean, invstd, sums = ops.convbn_forward(
            x, list(weights), geo, relu, gamma, beta,
            bn.running_mean if track else None, bn.running_var if track else None,
            bn.num_batches_tracked if track else None,
            float(bn.momentum) if bn.momentum is not None else 0.0, float(bn.eps), add,
            relu_out)
        # (beta only for the ReLU mask of relu_out, re-derived from z in the backward; with a
        # node sum the mask comes from the saved output instead: relu(bn(z) + add))
        out_mask = relu_out and add is not None
        ctx.save_for_backward(x, z, mean, invstd, sums, gamma,
                              beta if relu_out and not out_mask else None,
                              y if out_mask else None, *weights)
        ctx.relu_out = relu_out and not out_mask
        ctx.params = (gamma, beta) + weights  # gradient-accumulation fusion (ops/gradacc.py)
        ctx.caches = caches
        ctx.geo = geo
        ctx.relu = relu
        ctx.has_add = add is not None
        ctx.n_weights = len(weights)
        ctx.sink_in, ctx.sink_out = sinks  # (accumulate from / deposit the add's gradient)
        return y

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        x, z, mean, invstd, sums, gamma, beta, y, *weights = ctx.saved_tensors
        masked = None
        if y is not None:
            # relu(bn(z) + add): the gradient of both terms, masked once -- by the BatchNorm
            # backward kernel, which also writes the masked gradient (the add's) to `masked`
            masked = torch.empty_like(z)
        need_dx = ctx.needs_input_grad[0]
        fused = [gradacc.target(p) for p in ctx.params]
        # the backward-data GEMM reads W^T: transposed once per step, not per micro-batch
        wts = [c.get_transposed(w) for c, w in zip(ctx.caches, weights)] if need_dx else []
        ops = _ext.require(dy)
        side = _wgrad_stream(dy.device) if all(f for f, _ in fused[2:]) else None
        # deferred split weight gradients (ops/gradacc.py): per-parameter slabs
        slabs: List[Optional[Tensor]] = []
        firsts: List[int] = []
        for (fuse, _), w in zip(fused[2:], ctx.params[2:]):
            sb, first = gradacc.slab(w) if fuse else (None, False)
            slabs.append(sb)
            firsts.append(int(first))
        if all(sb is None for sb in slabs):
            slabs, firsts = [], []
        dx_into = None
        if ctx.sink_in is not None and ctx.sink_in.grad is not None:
            dx_into, ctx.sink_in.grad = ctx.sink_in.grad, None
            if not need_dx:
                dx_into = None
        dx, dgamma, dbeta, *dws = ops.convbn_backward(
            dy, x, z, mean, invstd, sums, gamma, weights, ctx.geo, ctx.relu, need_dx,
            [into for _, into in fused], wts, side is not None, slabs, firsts, beta,
            ctx.relu_out, dx_into, y, masked)
        if masked is not None:
            dy = masked
        dadd = dy if ctx.has_add and ctx.needs_input_grad[1] else None
        if dadd is not None and ctx.sink_out is not None:
            ctx.sink_out.grad = dadd  # the reader's backward adds it (see GradSink)
            dadd = None
        ctx.sink_in = ctx.sink_out = None
        if side is not None:
            # weight gradients on the side stream (written into .grad by the kernels)
            dz = dws[0]
            side.wait_stream(torch.cuda.current_stream(dy.device))
            dz.record_stream(side)
            x.record_stream(side)
            with torch.cuda.stream(side):
                dws = ops.convbn_wgrad(dz, x, weights, ctx.geo, ctx.relu,
                                       [into for _, into in fused[2:]], slabs, firsts)
        grads = [dgamma, dbeta] + dws
        for k, ((fuse, into), p) in enumerate(zip(fused, ctx.params)):
            if fuse:  # written into p.grad (or its slab) by the kernels
                if k >= 2 and slabs and gradacc.deferred(p, slabs[k - 2], grads[k]):
                    pass
                elif into is None:
                    gradacc.commit(p, grads[k])
                grads[k] = None
        del ctx.params, ctx.caches
        dgamma, dbeta, *dws = grads
        return (dx if need_dx else None, dadd,
                dgamma if ctx.needs_input_grad[2] else None,
                dbeta if ctx.needs_input_grad[3] else None, None, None, None, None, None, None,
                *dws)


def relu_conv_bn(x: Tensor, convs: Sequence[Tuple[nn.Conv2d, int]], bn: nn.BatchNorm2d,
                 relu: bool = True, add: Optional[Tensor] = None,
                 relu_out: bool = False, sink_in: Optional[GradSink] = None,
                 sink_out: Optional[GradSink] = None) -> Tensor:
    """``bn(cat([conv(relu(x) shifted by offset) for conv, offset in convs]))`` (+ ``add``),
    followed by a ReLU when ``relu_out`` (ResNet's Conv-BN-ReLU, and with ``add`` its
    residual join ``relu(bn(conv3(x)) + identity)`` in the same normalise pass).

    ``convs`` are ``(conv, offset)`` pairs whose outputs are concatenated on channels
    (one pair for ReLU-Conv-BN, two for FactorizedReduce: offsets 0 and 1).  Runs the
    fused HIP op when :func:`fusable`; callers check that first.
    """
    geo: List[int] = []
    for conv, offset in convs:
        # (the module's geometry, built once per offset: every micro-batch asks)
        cached = conv.__dict__.get('_convbn_geo')
        if cached is None or cached[0] != offset:
            cached = conv.__dict__['_convbn_geo'] = (offset, _geo(conv, offset))
        geo += cached[1]
    weights = [conv.weight for conv, _ in convs]
    return _ConvBN.apply(x, add, bn.weight, bn.bias, bn, geo, relu, relu_out,
                         [_weight_cache(conv) for conv, _ in convs], (sink_in, sink_out),
                         *weights)


def _weight_cache(conv: nn.Module) -> _TransformCache:
    """The module's step-scoped cache of derived weights (here: the transposed weight)."""
    cache = conv.__dict__.get('_wt_cache')
    if cache is None:
        cache = _TransformCache()
        conv.__dict__['_wt_cache'] = cache
    return cache


_LIMIT = (1 << 31) - 64  # 32-bit buffer offsets of the kernels


def fusable(x: Tensor, convs: Sequence[nn.Conv2d], bn: nn.Module) -> bool:
    if not (_ENABLED and _bn_ok(bn, x)):
        return False
    numel = x.numel()
    if numel * 4 >= _LIMIT:
        return False
    co = 0
    for c in convs:
        # the module's own configuration, checked once (every micro-batch asks)
        ok = c.__dict__.get('_fusable_conv')
        if ok is None:
            ok = c.__dict__['_fusable_conv'] = (conv_supported(c)
                                                and c.weight.numel() * 4 < _LIMIT)
        w = c.weight
        if not ok or w.dtype != torch.float32 or not w.is_cuda:
            return False
        co += c.out_channels
    return numel // max(1, x.shape[1]) * co * 4 < _LIMIT and _ext.available()


def fused_triplets(seq: nn.Sequential) -> Optional[List[Tuple[bool, nn.Conv2d, nn.BatchNorm2d]]]:
    """Split ``seq`` into (relu?, conv, bn) triplets, or ``None`` if it is not such a chain."""
    mods = list(seq.children())
    out: List[Tuple[bool, nn.Conv2d, nn.BatchNorm2d]] = []
    i = 0
    while i < len(mods):
        relu = isinstance(mods[i], nn.ReLU)
        j = i + 1 if relu else i
        if j + 1 >= len(mods) or not isinstance(mods[j], nn.Conv2d) or \
                not isinstance(mods[j + 1], nn.BatchNorm2d):
            return None
        out.append((relu, mods[j], mods[j + 1]))
        i = j + 2
    return out


class FusedChain(nn.Sequential):
    """A chain of (ReLU, Conv2d, BatchNorm2d) triplets run as fused ops.

    Children are the plain modules (the reference's state-dict keys); any triplet
    the fused op does not cover (biased / grouped / dilated convolutions, eval-mode
    BatchNorm, CPU tensors) runs eagerly.  ``add`` is folded into the last
    triplet's normalisation pass.
    """

    def forward(self, x: Tensor, add: Optional[Tensor] = None,  # type: ignore[override]
                start: int = 0) -> Tensor:
        """The chain from triplet ``start`` on (``start`` > 0: ``x`` is the output of
        triplet ``start - 1``, e.g. computed by :func:`group_relu_conv_bn`)."""
        triplets = self._triplets()
        if triplets is None:
            assert start == 0, 'start > 0 needs a chain of (ReLU, Conv2d, BatchNorm2d) triplets'
            out = super().forward(x)
            return out if add is None else out + add
        last = len(triplets) - 1
        for k, (relu, conv, bn) in enumerate(triplets):
            if k < start:
                continue
            extra = add if k == last else None
            if fusable(x, [conv], bn):
                x = relu_conv_bn(x, [(conv, 0)], bn, relu=relu, add=extra)
            else:
                x = bn(conv(F.relu(x) if relu else x))
                if extra is not None:
                    x = x + extra
        return x


    def _triplets(self) -> Optional[List[Tuple[bool, nn.Conv2d, nn.BatchNorm2d]]]:
        """:func:`fused_triplets` of this chain, cached while its children stay the same
        objects (every forward of every micro-batch asks)."""
        mods = tuple(self._modules.values())
        hit = self.__dict__.get('_triplet_cache')
        if hit is not None and len(hit[0]) == len(mods) and \
                all(a is b for a, b in zip(hit[0], mods)):
            return hit[1]
        triplets = fused_triplets(self)
        self.__dict__['_triplet_cache'] = (mods, triplets)
        return triplets


class ReLUConvBN(FusedChain):
    """``nn.Sequential(ReLU, Conv2d, BatchNorm2d)`` running as one fused op."""


# -- grouped ReLU-Conv-BN operations reading one input ------------------------------------

# TGPIPE_GROUP_CONVBN=0 runs grouped operations one by one.
_GROUP_ENABLED = os.environ.get('TGPIPE_GROUP_CONVBN', '1') != '0'


class _GroupCache:
    """The concatenated weights of a group (and their transpose) for one pipeline step:
    keyed like the Winograd transforms (storage, version, step of every weight)."""

    __slots__ = ('key', 'cat', 'cat_t', 'weights', 'ready', '__weakref__')

    def __init__(self) -> None:
        from torchgpipe_amd.ops.conv import cache_created
        cache_created()
        self.key: Optional[Tuple] = None
        self.cat: Optional[Tensor] = None
        self.cat_t: Optional[Tensor] = None
        self.weights: List[Tensor] = []  # detached aliases (see _TransformCache)
        self.ready: Optional[object] = None

    @staticmethod
    def _key(weights: Sequence[Tensor]) -> Tuple:
        from torchgpipe_amd.ops import conv as _conv
        return tuple((w.data_ptr(), w._version) for w in weights) + (_conv._STEP,)

    def get(self, weights: Sequence[Tensor]) -> Tuple[Tensor, Tensor]:
        from torchgpipe_amd.ops.conv import _await, _ready_event
        key = self._key(weights)
        if key != self.key or self.cat is None or self.cat_t is None:
            with torch.no_grad():
                cat = torch.cat([w.detach().reshape(w.shape[0], -1) for w in weights])
                self.cat = cat.view(cat.shape[0], cat.shape[1], 1, 1)
                self.cat_t = cat.t().contiguous().view(cat.shape[1], cat.shape[0], 1, 1)
            self.key = key
            self.weights = [w.detach() for w in weights]
            self.ready = _ready_event(self.cat_t)
        else:
            _await(self.cat, self.ready)
        return self.cat, self.cat_t

    def refresh(self) -> None:
        """Recompute the concatenations in place (same buffers) for this step."""
        weights = self.weights
        if not weights or self.cat is None or self.cat_t is None:
            return
        key = self._key(weights)
        if key != self.key:
            with torch.no_grad():
                flat = self.cat.view(self.cat.shape[0], self.cat.shape[1])
                torch.cat([w.reshape(w.shape[0], -1) for w in weights], out=flat)
                self.cat_t.view(flat.shape[1], flat.shape[0]).copy_(flat.t())
            self.key = key
        self.ready = None

    def __deepcopy__(self, memo: Dict[int, object]) -> '_GroupCache':
        return type(self)()  # derived data (see _TransformCache)

    def __reduce__(self) -> Tuple[object, ...]:
        return (type(self), ())


class _GroupConvBN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, bns: List[nn.BatchNorm2d], cache: _GroupCache,  # type: ignore[override]
                n_ops: int, *params: Tensor) -> Tuple[Tensor, ...]:
        weights = list(params[:n_ops])
        gammas, betas = list(params[n_ops:2 * n_ops]), list(params[2 * n_ops:])
        w_cat, _ = cache.get(weights)
        channels = [w.shape[0] for w in weights]
        track = [bn.track_running_stats and bn.running_mean is not None for bn in bns]
        outs = _ext.require(x).convbn_group_forward(
            x, w_cat, [1, 1, 1, 1, 0, 0, 0, 0], True, channels, gammas, betas,
            [bn.running_mean if t else None for bn, t in zip(bns, track)],
            [bn.running_var if t else None for bn, t in zip(bns, track)],
            [bn.num_batches_tracked if t else None for bn, t in zip(bns, track)],
            float(bns[0].momentum), float(bns[0].eps))
        ys, (z, mean, invstd) = outs[:n_ops], outs[n_ops:]
        ctx.save_for_backward(x, z, mean, invstd, *weights, *gammas)
        ctx.params = tuple(params)
        ctx.cache = cache
        ctx.channels = channels
        ctx.n_ops = n_ops
        return tuple(ys)

    @staticmethod
    def backward(ctx, *dys: Tensor):  # type: ignore[override]
        x, z, mean, invstd, *rest = ctx.saved_tensors
        n = ctx.n_ops
        weights, gammas = rest[:n], rest[n:]
        params = ctx.params
        # gradient-accumulation fusion per parameter (order: weights, gammas, betas)
        fused = [gradacc.target(p) for p in params]
        accum: List[Optional[Tensor]] = []
        for i in range(n):
            accum += [fused[n + i][1], fused[2 * n + i][1], fused[i][1]]
        slabs: List[Optional[Tensor]] = []
        firsts: List[int] = []
        for i in range(n):
            sb, first = gradacc.slab(params[i]) if fused[i][0] else (None, False)
            slabs.append(sb)
            firsts.append(int(first))
        if all(sb is None for sb in slabs):
            slabs, firsts = [], []
        need_dx = ctx.needs_input_grad[0]
        _, w_cat_t = ctx.cache.get(weights)
        out = _ext.require(x).convbn_group_backward(
            list(dys), x, z, mean, invstd, list(weights), w_cat_t, [1, 1, 1, 1, 0, 0, 0, 0],
            True, need_dx, ctx.channels, list(gammas), accum, slabs, firsts)
        dx = out[0]
        dgb, dws = out[1:1 + 2 * n], out[1 + 2 * n:]
        grads: List[Optional[Tensor]] = [None] * (3 * n)
        for i in range(n):
            grads[i] = dws[i]
            grads[n + i] = dgb[2 * i]
            grads[2 * n + i] = dgb[2 * i + 1]
        for k, ((fuse, into), p) in enumerate(zip(fused, params)):
            if fuse:  # written into p.grad (or its slab) by the kernels
                if k < n and slabs and gradacc.deferred(p, slabs[k], grads[k]):
                    pass
                elif into is None:
                    gradacc.commit(p, grads[k])  # type: ignore[arg-type]
                grads[k] = None
        del ctx.params, ctx.cache
        return (dx if need_dx else None, None, None, None, *grads)


def groupable(x: Tensor, triplets: Sequence[Tuple[bool, nn.Conv2d, nn.BatchNorm2d]]) -> bool:
    """Whether :func:`group_relu_conv_bn` takes these (relu, conv, bn) triplets: ReLU ->
    plain 1x1 convolutions of ``x`` -> BatchNorms with one momentum / eps, the grouped
    BatchNorm backward's channel size limit, and the fused-op conditions."""
    if not _GROUP_ENABLED or not 2 <= len(triplets) <= 3 or x.dim() != 4:
        return False
    bn0 = triplets[0][2]
    for relu, conv, bn in triplets:
        if not relu or tuple(conv.kernel_size) != (1, 1) or tuple(conv.stride) != (1, 1) or \
                tuple(conv.padding) != (0, 0) or not fusable(x, [conv], bn) or \
                bn.momentum != bn0.momentum or bn.eps != bn0.eps or \
                (bn.weight is None) != (bn0.weight is None) or \
                not bn.track_running_stats or bn.running_mean is None:
            return False
    if bn0.weight is None:
        return False
    co = sum(conv.out_channels for _, conv, _ in triplets)
    hw = x.shape[2] * x.shape[3]
    return bool(_ext.require(x).convbn_group_backward_ok(x.shape[0], co, hw)) and \
        x.numel() // max(1, x.shape[1]) * co * 4 < (1 << 31) - 64


def group_relu_conv_bn(x: Tensor, triplets: Sequence[Tuple[bool, nn.Conv2d, nn.BatchNorm2d]],
                       cache: '_GroupCache') -> Tuple[Tensor, ...]:
    """``[bn_i(conv_i(relu(x))) for each triplet]`` as one grouped op: one implicit-GEMM
    launch over the concatenated weights, one statistics / normalise pass writing each
    output, and one BatchNorm backward + one backward-data GEMM in the backward (callers
    check :func:`groupable` first)."""
    convs = [conv for _, conv, _ in triplets]
    bns = [bn for _, _, bn in triplets]
    params = ([c.weight for c in convs] + [b.weight for b in bns] + [b.bias for b in bns])
    return _GroupConvBN.apply(x, bns, cache, len(convs), *params)


# -- plain convolutions on the same implicit-GEMM kernels --------------------------------

def gemm_conv_eligible(x: Tensor, conv: nn.Conv2d) -> bool:
    """Convolutions the implicit-GEMM kernels take without BatchNorm: any kernel and
    stride, no bias / groups / dilation, fp32 on the GPU."""
    limit = (1 << 31) - 64  # 32-bit buffer offsets of the kernels
    out_numel = x.numel() // max(1, x.shape[1]) * conv.out_channels if x.dim() == 4 else 0
    return (_ENABLED and x.is_cuda and x.dtype == torch.float32 and x.dim() == 4
            and x.numel() * 4 < limit and conv.weight.numel() * 4 < limit
            and out_numel * 4 < limit
            and conv.weight.dtype == torch.float32 and conv.bias is None and conv.groups == 1
            and tuple(conv.dilation) == (1, 1) and conv.padding_mode == 'zeros'
            and isinstance(conv.padding, tuple) and _ext.available())


class _GemmConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, weight: Tensor, geo: List[int],  # type: ignore[override]
                cache: _TransformCache) -> Tensor:
        ctx.save_for_backward(x, weight)
        ctx.param = weight
        ctx.cache = cache
        ctx.geo = geo
        return _ext.require(x).conv_gemm_forward(x, weight, geo, False)

    @staticmethod
    def backward(ctx, dz: Tensor):  # type: ignore[override]
        x, weight = ctx.saved_tensors
        ops = _ext.require(dz)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = ops.conv_gemm_backward_data(dz, x, weight, ctx.geo, False,
                                             ctx.cache.get_transposed(weight))
        if ctx.needs_input_grad[1]:
            fuse, into = gradacc.target(ctx.param)
            sb, first = gradacc.slab(ctx.param) if fuse else (None, False)
            dw = ops.conv_gemm_backward_weight(dz, x, weight, ctx.geo, False, into, sb, first)
            if fuse:  # accumulated into / stored as weight.grad (ops/gradacc.py)
                if sb is not None and gradacc.deferred(ctx.param, sb, dw):
                    pass
                elif into is None:
                    gradacc.commit(ctx.param, dw)
                dw = None
        # a repeated backward (retain_graph=True) returns dw to autograd instead
        ctx.param = None
        return dx, dw, None, None


def gemm_conv2d(x: Tensor, conv: nn.Conv2d) -> Tensor:
    """``conv(x)`` on the implicit-GEMM MFMA kernels (caller checks eligibility)."""
    return _GemmConv.apply(x, conv.weight, _geo(conv), _weight_cache(conv))


class GemmConv2d(nn.Conv2d):
    """``nn.Conv2d`` whose GPU fp32 path is the implicit-GEMM MFMA kernel (no MIOpen)."""

    def forward(self, input: Tensor) -> Tensor:
        if gemm_conv_eligible(input, self):
            return gemm_conv2d(input, self)
        return super().forward(input)
