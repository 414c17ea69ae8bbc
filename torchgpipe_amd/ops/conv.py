"""3×3 convolution on the CDNA4 matrix cores: Winograd F(4×4, 3×3) / F(2×2, 3×3) with f32 MFMA.

:class:`WinogradConv2d` is a drop-in ``nn.Conv2d`` (same parameters, same
state-dict keys) whose 3×3 / stride 1 / pad 1 / fp32 GPU forward and
backward-data run the fused HIP kernels of ``csrc/winograd_f4.hip`` (planes ≥ 8²)
and ``csrc/winograd.hip`` (smaller planes); the weight
gradient runs the F(4x4) / F(2x2) Winograd wgrad kernels wherever they beat MIOpen's
wrw (see ``_wgrad_f4`` and ``_wgrad_on_mfma``).
Other configurations, CPU tensors and non-fp32 dtypes use ``F.conv2d``.

The Winograd-domain weights ``U = G g Gᵀ`` (and the rotated/transposed ``U'``
of backward-data) are cached per parameter version *and pipeline step*: a step
runs the same weights over every micro-batch (forward, recompute, backward), so
the transform runs once per optimizer step instead of once per call.

* Staleness: the key includes a step counter that ``GPipe.forward`` /
  ``PipelineStage.forward`` advance (:func:`new_step`), so weights changed
  between steps through ``param.data`` (which does not bump ``_version``), EMA
  swaps or manual surgery are always re-transformed; :func:`clear_winograd_caches`
  drops a module's caches explicitly.
* Refresh in place: :func:`refresh_step_caches` (``PipelineStage.forward``, once per step,
  on the stage's main stream) recomputes every existing entry *into its own buffer*, so a
  cached transform keeps its address across steps -- which captured cell graphs
  (``parallel/segments.py``) rely on -- and is ordered before every lane that later reads
  it.  An entry created lazily inside a step records an event, and a reader on another
  stream waits for it (forward lanes: micro-batch 1 may reach a layer before micro-batch 0
  has transformed its weights).
* Memory: every cached byte counts against a per-device budget.  A pipeline stage sizes it
  from its own first step, which runs uncached (:func:`size_cache_budget`,
  ``PipelineStage``): afterwards the cache may use half of the device memory that step
  left free, capped at 5 % of the device -- it only ever takes memory the stage does not
  need, so it cannot make a model that fits uncached run out of memory (the largest
  trainable model is the cache-free one).  ``TGPIPE_WINOGRAD_CACHE_FRACTION=f`` is the
  memory-lean mode: at most ``f`` times the first step's peak (``benchmarks/memory.py``
  uses 0.15, so a stage grows by at most 15 %; the speed benchmarks' stages would then
  recompute part of their transforms per call).  Before a stage has sized it (or outside
  a stage) the budget is 5 % of the device; ``TGPIPE_WINOGRAD_CACHE_MB`` overrides all of
  these.  A transform that would exceed the budget is used for the call and dropped.
"""
import os
import threading
from typing import Any, Dict, List, Optional, Sequence, Tuple
import weakref

import torch
from torch import Tensor, nn
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext, gradacc

__all__ = ['WinogradConv2d', 'winograd_conv2d', 'wino_eligible', 'new_step',
           'clear_winograd_caches', 'cache_bytes', 'refresh_step_caches', 'hold_cache',
           'size_cache_budget', 'conv_with_bn_stats']

_STEP = 0
_CACHE_BYTES: Dict[torch.device, int] = {}  # cached bytes per device
_BUDGET: Optional[int] = None
# per-device budgets set by size_cache_budget / hold_cache (bytes)
_DEVICE_BUDGET: Dict[torch.device, int] = {}
_FRACTION = os.environ.get('TGPIPE_WINOGRAD_CACHE_FRACTION')
CACHE_PEAK_FRACTION: Optional[float] = float(_FRACTION) if _FRACTION else None
# the implicit-GEMM pre-split weights' budget cap, MiB (csrc/convbn.cpp presplit_budget)
PRESPLIT_MB = max(0, int(os.environ.get('TGPIPE_CG_PRESPLIT_MB', '2048')))


def new_step() -> None:
    """Start a new pipeline step: every cached weight transform is re-validated, and the
    ``AccumulateGrad`` nodes pinned by the previous step's fused backward are released
    (``ops/gradacc.py``), so this step's graph gets nodes bound to its own streams."""
    global _STEP
    _STEP += 1
    if _ext._loaded:
        # the implicit GEMMs' pre-split weights too (csrc/convbn.cpp presplit_of): an
        # update through ``param.data`` moves no version counter
        torch.ops.tgpipe.conv_gemm_presplit_step(_STEP)
    from torchgpipe_amd.ops import gradacc
    gradacc.release()


def cache_bytes() -> int:
    """Bytes currently held by Winograd weight-transform caches (this process)."""
    return sum(_CACHE_BYTES.values())


def _device_cap(device: torch.device) -> int:
    return torch.cuda.get_device_properties(device).total_memory // 20


def _budget(device: torch.device) -> int:
    global _BUDGET
    mb = os.environ.get('TGPIPE_WINOGRAD_CACHE_MB')
    if mb is not None:
        if _BUDGET is None:
            _BUDGET = int(float(mb) * (1 << 20))
        return _BUDGET
    sized = _DEVICE_BUDGET.get(device)
    return sized if sized is not None else _device_cap(device)


def hold_cache(device: torch.device) -> None:
    """Cache nothing on ``device`` (a stage's first step, which measures its footprint) --
    nor pre-split implicit-GEMM weights (csrc/convbn.cpp presplit_of)."""
    _DEVICE_BUDGET[device] = 0
    _presplit_budget(0)


def _presplit_budget(mb: int) -> None:
    """The implicit-GEMM pre-split weights' budget (MiB; -1: ``TGPIPE_CG_PRESPLIT_MB``)."""
    global presplit_budget_mb
    presplit_budget_mb = mb
    if _ext.available():
        torch.ops.tgpipe.conv_gemm_presplit(mb, False)


# the last pre-split budget set from here (MiB; -1 = the environment's default)
presplit_budget_mb = -1


def size_cache_budget(device: torch.device, peak_bytes: int,
                      fraction: Optional[float] = None) -> int:
    """Size the caches on ``device`` from a stage's uncached step peak ``peak_bytes``: half
    the memory that leaves free, or (``fraction`` / ``TGPIPE_WINOGRAD_CACHE_FRACTION``)
    that fraction of the peak; at most 5 % of the device.  Returns the budget."""
    fraction = CACHE_PEAK_FRACTION if fraction is None else fraction
    if fraction is not None:
        budget = int(fraction * peak_bytes)
    else:
        total = torch.cuda.get_device_properties(device).total_memory
        budget = max(0, total - peak_bytes) // 2
    budget = min(_device_cap(device), budget)
    _DEVICE_BUDGET[device] = budget
    # pre-split implicit-GEMM weights (1.5x the weights they split): off in the memory-lean
    # mode (a fraction of the peak, e.g. benchmarks/memory.py); else their own budget
    # (TGPIPE_CG_PRESPLIT_MB), capped by half of what the measuring step and the transform
    # cache leave free -- like the transform cache, memory the stage did not need
    if fraction is not None:
        _presplit_budget(0)
    else:
        total = torch.cuda.get_device_properties(device).total_memory
        left = max(0, total - peak_bytes - budget) // 2
        _presplit_budget(min(PRESPLIT_MB, left >> 20))
    return budget


def _derive(weight: Tensor, slot: Tuple, out: Optional[Tensor] = None) -> Tensor:
    """The derived weight of one cache slot: ``(flip, f4, bg)`` Winograd transforms, or
    ``(True, True, 'T')`` the ``[ci][co][kh][kw]`` transpose -- written into ``out`` when
    given (the per-step refresh: one pass over the transform, not a new one and a copy;
    U-Net(5,64)'s transforms are ~7 GB per step)."""
    with torch.no_grad():
        w = weight.detach()
        if slot[2] == 'T':
            if out is not None:
                return out.copy_(w.transpose(0, 1))
            return w.transpose(0, 1).contiguous()
        ops = _ext.require(weight)
        flip, f4, bg = slot
        w = w.contiguous()
        if bg:
            return ops.bg_weight(w, flip, bg, out)
        return ops.wino4_weight(w, flip, out) if f4 else ops.wino_weight(w, flip, out)


def _ready_event(t: Tensor) -> Optional[Any]:
    """An event after the work that produced ``t`` on the current stream (``None`` on CPU or
    inside a capture, where every reader is ordered by the capture itself)."""
    if not t.is_cuda or torch.cuda.is_current_stream_capturing():
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(t.device))
    return ev


def _await(t: Tensor, ready: Optional[Any]) -> None:
    if ready is not None and not torch.cuda.is_current_stream_capturing():
        torch.cuda.current_stream(t.device).wait_event(ready)


# guards the miss path of every _TransformCache (derive + insert + byte accounting)
_CACHE_LOCK = threading.RLock()


class _TransformCache:
    """Derived weights keyed by (storage, version, device, step) of the parameter.

    Entries per slot ``(flip, f4, bg)``: F(2x2) ``U[Rp][Op][16]``, F(4x4)
    ``U4[Rp/4][Op/16][4][16][36]``, the batched-GEMM layouts, or the transpose (slot
    ``(True, True, 'T')``).  Each entry is ``(key, tensor, ready event)``.
    """

    __slots__ = ('_entries', '_weight', '__weakref__')

    def __init__(self) -> None:
        cache_created()
        self._entries: Dict[Tuple, Tuple[Tuple[int, int, torch.device, int], Tensor,
                                         Optional[Any]]] = {}
        # a detached alias of the weight (same storage and version counter): the caller may
        # pass a saved-tensor object rather than the parameter, which a weak reference
        # would not keep
        self._weight: Optional[Tensor] = None

    def _lookup(self, weight: Tensor, slot: Tuple) -> Tensor:
        dev = weight.device
        key = (weight.data_ptr(), weight._version, dev, _STEP)
        hit = self._entries.get(slot)
        if hit is not None and hit[0] == key:
            _await(hit[1], hit[2])
            return hit[1]
        if weight.is_cuda and torch.cuda.is_current_stream_capturing():
            # Inside a hipGraph capture the cache is read, never written: an entry created
            # here would live in that graph's private pool with no ready event, and another
            # graph replayed on another lane could hit it before this graph has run (a
            # stage with one warm-up step captures before any cached step).  The graph
            # derives its own copy on every replay instead.
            return _derive(weight, slot)
        with _CACHE_LOCK:  # (PipelineStage(backward_thread=True): two host threads)
            hit = self._entries.get(slot)
            if hit is not None and hit[0] == key:
                _await(hit[1], hit[2])
                return hit[1]
            if hit is not None:  # stale: release before transforming again
                _CACHE_BYTES[dev] -= hit[1].numel() * hit[1].element_size()
                del self._entries[slot]
            u = _derive(weight, slot)
            size = u.numel() * u.element_size()
            if _CACHE_BYTES.get(dev, 0) + size <= _budget(dev):
                self._entries[slot] = (key, u, _ready_event(u))
                self._weight = weight.detach()
                _CACHE_BYTES[dev] = _CACHE_BYTES.get(dev, 0) + size
            return u

    def get(self, weight: Tensor, flip: bool, f4: bool = False, bg: int = 0) -> Tensor:
        """The transformed weight for ``flip`` (backward-data) and the kernel family:
        F(2x2) (default), F(4x4) fused (``f4``) or the batched-GEMM layout of F(4x4) /
        F(2x2) (``bg`` = 4 / 2)."""
        return self._lookup(weight, (flip, f4, bg))

    def get_transposed(self, weight: Tensor) -> Tensor:
        """``weight`` as ``[ci][co][kh][kw]`` (contiguous): the backward-data GEMM operand
        of the implicit-GEMM convolutions, transposed once per step instead of per call."""
        return self._lookup(weight, (True, True, 'T'))

    def refresh(self) -> None:
        """Recompute every entry in place for the weight's current value and this step."""
        weight = self._weight
        if weight is None:
            return
        key = (weight.data_ptr(), weight._version, weight.device, _STEP)
        for slot, (old, u, _) in list(self._entries.items()):
            if old[0] != key[0] or old[2] != key[2]:
                continue  # another weight storage (module surgery): left to the lazy path
            if old != key:
                _derive(weight, slot, out=u)
            self._entries[slot] = (key, u, None)

    def derived(self) -> List[Tensor]:
        """The cached derived weights (the tensors other caches may be keyed on)."""
        return [u for _, u, _ in self._entries.values()]

    def clear(self) -> None:
        for _, u, _ in self._entries.values():
            _CACHE_BYTES[u.device] -= u.numel() * u.element_size()
        self._entries.clear()
        self._weight = None

    def __del__(self) -> None:
        try:
            self.clear()
        except Exception:  # interpreter shutdown
            pass

    # derived data: a copied or pickled module starts with an empty cache (the entries hold
    # device tensors and HIP events of this process)
    def __deepcopy__(self, memo: Dict[int, Any]) -> '_TransformCache':
        return type(self)()

    def __reduce__(self) -> Tuple[Any, ...]:
        return (type(self), ())


# bumped whenever a step-scoped cache object (_TransformCache, convbn._GroupCache) is made:
# refresh_step_caches re-scans a module's attributes only then
_CACHE_EPOCH = 0


def cache_created() -> None:
    global _CACHE_EPOCH
    _CACHE_EPOCH += 1


# module -> (cache epoch, weak references to its cache objects); outside the module, so
# pickling or copying a module carries none of it
_SCANS: 'weakref.WeakKeyDictionary[nn.Module, Tuple[int, List[Any]]]' = \
    weakref.WeakKeyDictionary()


def _step_caches(module: nn.Module) -> List[Any]:
    """The cache objects held by ``module``'s (sub)modules: scanned once per cache epoch (a
    ResNet-101 scan is ~2.5 ms of host time at every step start otherwise)."""
    from torchgpipe_amd.ops.convbn import _GroupCache
    hit = _SCANS.get(module)
    if hit is None or hit[0] != _CACHE_EPOCH:
        refs = [weakref.ref(v) for m in module.modules() for v in list(vars(m).values())
                if isinstance(v, (_TransformCache, _GroupCache))]
        hit = _SCANS[module] = (_CACHE_EPOCH, refs)
    return [v for v in (r() for r in hit[1]) if v is not None]


def refresh_step_caches(module: nn.Module) -> None:
    """Refresh every step-scoped derived-weight cache in ``module`` in place (current
    stream): Winograd transforms, transposed weights, grouped-GEMM concatenations and the
    split-bf16 GEMMs' pre-split weights."""
    sources: List[Tensor] = []
    for v in _step_caches(module):
        v.refresh()
        if isinstance(v, _TransformCache):
            sources += v.derived()
        else:
            sources += [t for t in (v.cat, v.cat_t) if t is not None]
    if _ext._loaded:
        # then the implicit-GEMM kernels' pre-split weights (csrc/convbn.cpp presplit_of)
        # derived from this module's parameters and the transposes / concatenations above
        sources += [p for p in module.parameters() if p.is_cuda]
        if sources:
            torch.ops.tgpipe.conv_gemm_presplit_refresh(sources)


def clear_winograd_caches(module: torch.nn.Module) -> None:
    """Drop the cached weight transforms of every WinogradConv2d (and the transposed
    weights of the implicit-GEMM convolutions) in ``module``."""
    for m in module.modules():
        for attr in ('_wino', '_wt_cache'):
            cache = getattr(m, attr, None)
            if isinstance(cache, _TransformCache):
                cache.clear()


# Winograd F(4x4,3x3) (csrc/winograd_f4.hip) on planes of at least this size; F(2x2) on
# smaller ones.  benchmarks/wino_variants.py (profiles/wino_f4_variants.json): F(4x4)
# 1.17-1.45x faster than F(2x2) from 12^2 up, slower at 6^2 (a 4x4 tile wastes 5/9 of a
# 6-pixel plane).  The F(4x4) kernel's 32-bit offsets need the input below 1 GiB.
F4_MIN_PLANE = 8
# Fused F(4x4) forward / backward-data kernel for < 512 channels: 6 (slab one step ahead)
# or 18 (slab ring, two steps ahead; csrc/winograd_f4.hip).  TGPIPE_F4_FUSED_VARIANT.
_F4_FUSED_VARIANT = int(os.environ.get('TGPIPE_F4_FUSED_VARIANT', '6'))
F4_MAX_BYTES = (1 << 30) - 64


# 6x6 planes (U-Net's bottom level) waste 5/9 of a 4x4-tile grid, so F(4x4) spends as
# many multiplies there as F(2x2); with >= 512 channels its non-fused GEMM still wins
# (profiles/wino_f4_6x6.json: forward 0-15 %, weight gradient 10-17 %).
F4_MIN_PLANE_WIDE = 6
F4_WIDE_CHANNELS = 512


# The F(4x4) weight cache holds 36 floats per (in, out) channel pair and direction (8x
# the weight, vs 3.6x for F(2x2)): layers whose cache would pass this stay on F(2x2), so
# memory-bound giant models (benchmarks/memory.py: U-Net(48,576)'s 18432-channel
# bottleneck, 49 GB per direction in F(4x4)) keep their measured footprint.
F4_MAX_CACHE_BYTES = 2 << 30
# TGPIPE_WINOGRAD_F4=0 keeps every layer on F(2x2).
F4_ENABLED = os.environ.get('TGPIPE_WINOGRAD_F4', '1') != '0'


def _use_f4(x: Tensor, out_channels: int = 0) -> bool:
    if not F4_ENABLED or x.shape[1] * out_channels * 36 * 4 > F4_MAX_CACHE_BYTES:
        return False
    plane = min(x.shape[2], x.shape[3])
    # forward at 6x6: ahead at 16 images (0.30 vs 0.36 ms), even at 40 (0.67 vs 0.66)
    wide = (plane >= F4_MIN_PLANE_WIDE and out_channels >= F4_WIDE_CHANNELS
            and x.shape[1] >= F4_WIDE_CHANNELS and x.shape[0] <= 24)
    return (plane >= F4_MIN_PLANE or wide) and x.numel() * x.element_size() < F4_MAX_BYTES


# Batched-GEMM Winograd (csrc/winograd_f4.hip bg_*: input-transform pass, 36 / 16 independent
# 128 x 48-128 MFMA GEMMs, output-transform pass) for convolutions with >= 256 channels on
# both sides: 1.1-1.9x faster than the fused / non-fused F(4x4) kernels and the F(2x2)
# kernel on every such U-Net shape at 16-40 images (benchmarks/bg_bench.py,
# profiles/r3/bg_bench.json), F(2x2) on 6x6 planes (a 4x4 tile grid wastes 5/9 there).
# TGPIPE_WINOGRAD_BG=0 keeps the older kernels.
BG_ENABLED = os.environ.get('TGPIPE_WINOGRAD_BG', '1') != '0'
BG_MIN_CHANNELS = int(os.environ.get('TGPIPE_WINOGRAD_BG_MIN_CHANNELS', '256'))


def _bg_kind(x: Tensor, out_channels: int) -> int:
    """4 (F(4x4)), 2 (F(2x2)) or 0 (not the batched-GEMM path) for this convolution."""
    r = x.shape[1]
    plane = min(x.shape[2], x.shape[3])
    if not BG_ENABLED or r < BG_MIN_CHANNELS or out_channels < BG_MIN_CHANNELS or plane < 6:
        return 0
    kind = 2 if plane < 8 else 4
    positions = 16 if kind == 2 else 36
    if r * out_channels * positions * 4 > F4_MAX_CACHE_BYTES or \
            x.numel() * x.element_size() >= F4_MAX_BYTES:
        return 0
    tiles = x.shape[0] * -(-x.shape[2] // kind) * -(-x.shape[3] // kind)
    # the GEMM's padded operands and products (positions x channels x tiles) stay in the
    # kernels' 32-bit index range
    if positions * max(r, out_channels) * (tiles + 192) >= (1 << 31):
        return 0
    return kind


def _conv(x: Tensor, cache: _TransformCache, weight: Tensor, bias: Optional[Tensor],
          flip: bool) -> Tensor:
    """One Winograd convolution launch: forward (flip=False) or backward-data (flip=True)."""
    ops = _ext.require(x)
    out_channels = weight.shape[1] if flip else weight.shape[0]
    kind = _bg_kind(x, out_channels)
    if kind:
        return ops.bg_conv(x, cache.get(weight, flip, bg=kind), bias, out_channels, 0, 0, kind)
    if _use_f4(x, out_channels):
        # 32-channel workgroups (variant 7) when a 64-channel one (variant 6) would idle
        # half its waves, or when the 64-channel grid covers well under one workgroup per
        # CU (before split-K): profiles/wino_f4_variants.json, 16 images at 12^2 / 24^2
        # (80 / 144 blocks) 12 % / 10 % faster on 32 channels; 40 images at 12^2 (192
        # blocks) and every larger grid 3-14 % faster on 64.  Both copy the weight slab
        # with LDS-DMA (variants 4 / 5 stage it through registers: 2-12 % slower).
        # From 512 output channels the input transform runs as its own pass (variants 14 /
        # 15: V written once, then a GEMM kernel with both operands by LDS-DMA): 20-28 %
        # faster at 512-2048 channels, where V is re-read by >= 8 channel blocks; slower
        # on the wide planes with few channels (64 @ 192^2: 0.75 vs 0.52 ms).
        tiles = x.shape[0] * ((x.shape[2] + 3) // 4) * ((x.shape[3] + 3) // 4)
        blocks = -(-tiles // 32) * -(-out_channels // 64)
        if out_channels >= 512:
            # 6x6 planes: the 32-channel GEMM (0.67 vs 0.73 ms at 40 images)
            small = blocks < 160 or min(x.shape[2], x.shape[3]) < F4_MIN_PLANE
            variant = 15 if small else 14
        else:
            variant = 7 if out_channels <= 32 or blocks < 160 else _F4_FUSED_VARIANT
        return ops.wino4_conv(x, cache.get(weight, flip, True), bias, out_channels, variant)
    return ops.wino_conv(x, cache.get(weight, flip), bias, out_channels)


class _WinogradConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, weight: Tensor, bias: Optional[Tensor],  # type: ignore[override]
                cache: _TransformCache) -> Tensor:
        y = _conv(x.contiguous(), cache, weight, bias, False)
        ctx.save_for_backward(x, weight)
        ctx.cache = cache
        ctx.has_bias = bias is not None
        ctx.param = weight  # gradient-accumulation fusion (ops/gradacc.py)
        return y

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        dx, dw = _conv_grads(x, weight, dy, ctx.cache, ctx.needs_input_grad[0],
                             ctx.needs_input_grad[1], ctx.param)
        # a repeated backward (retain_graph=True) returns dw to autograd instead
        ctx.param = None
        db = None
        if ctx.has_bias and ctx.needs_input_grad[2]:
            db = dy.sum((0, 2, 3))
        return dx, dw, db, None


class _WinogradConvStats(torch.autograd.Function):
    """The batched-GEMM forward of :class:`_WinogradConv` whose output pass also leaves the
    BatchNorm (mean, M2) partials of its output (``bg_conv``'s ``stats``): a linked
    BatchNorm (``ops/fusion.py`` ``ConvBN2d``) normalises from them without its own
    statistics pass.  Backward as :class:`_WinogradConv`."""

    @staticmethod
    def forward(ctx, x: Tensor, weight: Tensor, cache: _TransformCache,  # type: ignore[override]
                kind: int) -> Tuple[Tensor, Tensor]:
        ops = _ext.require(x)
        x = x.contiguous()
        n, _, h, w = x.shape
        k = weight.shape[0]
        groups = -(-n // ops.bg_stats_images(n, h, w, kind))
        stats = torch.empty(2, groups, k, device=x.device, dtype=torch.float32)
        y = ops.bg_conv(x, cache.get(weight, False, bg=kind), None, k, 0, 0, kind,
                        stats=stats)
        ctx.save_for_backward(x, weight)
        ctx.cache = cache
        ctx.param = weight
        ctx.mark_non_differentiable(stats)
        # (no zero-filled gradient for `stats` per backward: one fill kernel per call)
        ctx.set_materialize_grads(False)
        return y, stats

    @staticmethod
    def backward(ctx, dy: Optional[Tensor], _dstats: Optional[Tensor]):  # type: ignore[override]
        if dy is None:
            ctx.param = None
            return None, None, None, None
        x, weight = ctx.saved_tensors
        dx, dw = _conv_grads(x, weight, dy.contiguous(), ctx.cache, ctx.needs_input_grad[0],
                             ctx.needs_input_grad[1], ctx.param)
        ctx.param = None
        return dx, dw, None, None


# TGPIPE_BG_BN_STATS=0: a linked BatchNorm after a batched-GEMM Winograd layer takes its own
# statistics pass (bn_stats_kernel) instead of the output pass's partials
BG_BN_STATS = os.environ.get('TGPIPE_BG_BN_STATS', '1') != '0'


def conv_with_bn_stats(module: nn.Conv2d, x: Tensor
                       ) -> Optional[Tuple[Tensor, Tensor, int]]:
    """``(y, stats, images per group)`` of a bias-free 3x3 ``WinogradConv2d`` on the
    batched-GEMM path, with its output's BatchNorm partials (``_WinogradConvStats``);
    ``None`` when the layer takes another path.  Callers checked ``wino_eligible``."""
    if not BG_BN_STATS or module.bias is not None:
        return None
    kind = _bg_kind(x, module.out_channels)
    if not kind:
        return None
    y, stats = _WinogradConvStats.apply(x, module.weight, module._wino, kind)
    n, _, h, w = x.shape
    return y, stats, _ext.require(x).bg_stats_images(n, h, w, kind)


def _conv_grads(x: Tensor, weight: Tensor, dy: Tensor, cache: _TransformCache, need_x: bool,
                need_w: bool, param: Optional[Tensor] = None
                ) -> Tuple[Optional[Tensor], Optional[Tensor]]:
    """Backward-data and weight gradient of the 3x3 / stride 1 / pad 1 convolution.

    With ``param`` (the weight as an autograd leaf) the Winograd weight-gradient kernels
    add straight into ``param.grad`` when autograd would accumulate there anyway
    (``ops/gradacc.py``): a GPipe step then spends no ``grad += new`` pass over the
    weights per micro-batch (U-Net p8's stage 3: 105 M parameters, 39 extra passes), and
    the parameter's AccumulateGrad node never runs, so micro-batches back-propagating on
    different streams (forward / recompute lanes) need no cross-stream sync for it.
    Returns ``dw = None`` when the kernels wrote the gradient themselves.
    """
    dx = dw = None
    if need_x:
        dx = _conv(dy, cache, weight, None, True)
    if need_w:
        ops = _ext.require(dy)
        f4, mfma = _wgrad_f4(x, dy, weight), _wgrad_on_mfma(x, weight)
        # the MIOpen weight gradient is accumulated here as well (one add), so no
        # AccumulateGrad node of these parameters runs: under forward / recompute lanes a
        # node shared by micro-batches of different streams would otherwise sync them
        fuse, into = gradacc.target(param) if param is not None else (False, None)
        if f4:
            dw = ops.wino4_wgrad(x, dy, 0, _wgrad_f4_variant(x, weight), into)
        elif mfma:
            dw = ops.wino_wgrad(x, dy, 0, -1, into)
        else:
            dw = torch.ops.aten.convolution_backward(
                dy, x, weight, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1,
                [False, True, False])[1]
        if fuse:
            assert param is not None
            if into is None:
                gradacc.commit(param, dw)
            elif not (f4 or mfma):  # the library result is a new tensor
                into.add_(dw)
            dw = None
    return dx, dw


# TGPIPE_WGRAD_EMU=0 keeps the F(4x4) weight gradients on the f32 matrix pipes.
WGRAD_EMU = os.environ.get('TGPIPE_WGRAD_EMU', '1') != '0'
# the split-bf16 batched GEMM (variant 2) from this many 4x4 tiles on: its [36][K][C]
# products go through HBM once, which only the longer tile reductions amortise
WGRAD_EMU_MIN_TILES = 320


def _wgrad_f4_variant(x: Tensor, weight: Tensor) -> int:
    """F(4x4) weight-gradient kernel (benchmarks/wgrad_variants.py,
    profiles/r5/wgrad_variants_emu.json): from 512 channels on both sides the non-fused
    kernels (transform passes + GEMM; 11-23 % faster than the fused one there, 1.2-3.6x
    slower on the wide shallow planes, profiles/wgrad_f4_variants.json) -- the split-bf16
    batched GEMM (2) once the tile count amortises its products' trip through HBM
    (40 x 512^2 at 24^2: 0.321 vs 0.401 ms; 40 x 1024^2 at 12^2: 0.286 vs 0.334), the f32
    one (1) below (16 x 2048^2 at 6^2: 0.294 vs 0.474).

    Round 6 (benchmarks/diag/wgrad_small_probe.py, profiles/r6/wgrad_small_probe.json): in
    isolation the non-fused kernel led by 3-14 % on ResNet-101's 256-channel 14^2 layers,
    but inside the stage (after the backward-data pass, with x / dy warm in L2) the fused
    kernel's 1792 dispatches plus the rest came to 125.9 ms of ResNet p4 stage 3's kernel
    time against 130.5 ms for the non-fused passes (profiles/r6/bg_input_cpt/
    p4_new_wgrad_rule.md), so the rule stayed as it was."""
    if min(weight.shape[0], weight.shape[1]) < 512:
        return 0
    tiles = x.shape[0] * -(-x.shape[2] // 4) * -(-x.shape[3] // 4)
    return 2 if WGRAD_EMU and tiles >= WGRAD_EMU_MIN_TILES else 1


def _wgrad_f4(x: Tensor, dy: Tensor, weight: Tensor) -> bool:
    """Weight gradient on the F(4x4,3x3) kernel (csrc/winograd_f4.hip).

    benchmarks/wgrad_variants.py (profiles/wgrad_f4_variants.json): 1.25-1.6x faster than
    the F(2x2) kernel and 1.6-2.4x faster than MIOpen's wrw on every U-Net shape from
    12^2 up (74-251 TFLOP/s direct-equivalent), on 32-channel layers too.  Below 16
    input channels the 32-wide channel block is mostly padding (the 3-channel input conv
    stays on MIOpen); 32-bit buffer offsets need both operands below 1 GiB.
    """
    plane = min(x.shape[2], x.shape[3])
    wide = min(weight.shape[0], weight.shape[1]) >= F4_WIDE_CHANNELS
    return (F4_ENABLED and weight.shape[1] >= 16
            and (plane >= F4_MIN_PLANE or (plane >= F4_MIN_PLANE_WIDE and wide))
            and x.numel() * x.element_size() < F4_MAX_BYTES
            and dy.numel() * dy.element_size() < F4_MAX_BYTES)


def _wgrad_on_mfma(x: Tensor, weight: Tensor) -> bool:
    """Weight gradient on the Winograd MFMA kernels where they beat MIOpen's wrw.

    benchmarks/wgrad_variants.py (profiles/wgrad_variants.json): the double-buffered
    64x64 kernel (variant 2) runs 133-170 TFLOP/s direct-equivalent on every U-Net
    shape with > 32 output channels (MIOpen wrw: 75-107); with <= 32 output channels
    the 64x32 kernel (variant 0) still wins on large planes with >= 64 input channels
    (128->32 @192^2: 1.13 vs 1.72 ms) and MIOpen wins the rest (32->32 @192^2).
    """
    k, c = weight.shape[0], weight.shape[1]
    if k > 32:
        return c >= 16
    return c >= 64 and x.shape[2] * x.shape[3] >= 96 * 96


# Below this many input channels the 8-channel reduction chunk is mostly padding
# and MIOpen's direct kernels win (U-Net's 3-channel input conv: 0.18 vs 0.24 ms).
MIN_CHANNELS = 8


# TGPIPE_WINOGRAD=0: every convolution on MIOpen (F.conv2d), no weight-transform caches.
WINOGRAD_ENABLED = os.environ.get('TGPIPE_WINOGRAD', '1') != '0'

# A layer whose F(2x2) weight transform (16 floats per channel pair, 1.78x the weight)
# would pass this stays on MIOpen: giant models (U-Net(48,576)'s 18432^2 bottleneck
# convolutions, 21.7 GB per transform) must not need a transient copy of that size.
MAX_TRANSFORM_BYTES = int(float(os.environ.get('TGPIPE_WINOGRAD_MAX_TRANSFORM_MB', '2048'))
                          * (1 << 20))


# A convolution whose weight transform dwarfs its input -- a few images through thousands
# of channels, e.g. benchmarks/memory.py's U-Net(48,160) at micro-batch 1 (2560 channels at
# 12^2: 943 MB of F(4x4) transform for a 1.5 MB input, ratio 640) -- stays on MIOpen: the
# transform would move far more bytes than the convolution reads, and when it is not
# cached it is a transient the size of the transform (U-Net(48,160) p8's fullest stage 33.6
# vs 22.4 GiB).  U-Net(5,64)'s deepest layers at 16 images per micro-batch reach 57.
WEIGHT_DOMINATED_RATIO = float(os.environ.get('TGPIPE_WINOGRAD_WEIGHT_RATIO', '256'))


def _transform_ratio(x: Tensor, weight: Tensor) -> float:
    """Weight-transform floats (16 / 36 per channel pair at F(2x2) / F(4x4) planes) per
    input float."""
    positions = 16 if min(x.shape[2], x.shape[3]) < F4_MIN_PLANE else 36
    return weight.shape[0] * weight.shape[1] * positions / max(1, x.numel())


def wino_eligible(x: Tensor, weight: Tensor, stride: Sequence[int] = (1, 1),
                  padding: Sequence[int] = (1, 1), dilation: Sequence[int] = (1, 1),
                  groups: int = 1) -> bool:
    """Whether the HIP Winograd kernel computes this convolution."""
    return (WINOGRAD_ENABLED and x.is_cuda and x.dim() == 4 and x.dtype == torch.float32
            and weight.shape[1] >= MIN_CHANNELS
            and weight.shape[0] * weight.shape[1] * 16 * 4 <= MAX_TRANSFORM_BYTES
            and weight.dtype == torch.float32 and tuple(weight.shape[2:]) == (3, 3)
            and tuple(stride) == (1, 1) and tuple(padding) == (1, 1)
            and tuple(dilation) == (1, 1) and groups == 1
            and _transform_ratio(x, weight) <= WEIGHT_DOMINATED_RATIO)


def winograd_conv2d(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None,
                    cache: Optional[_TransformCache] = None) -> Tensor:
    """``F.conv2d(x, weight, bias, padding=1)`` for 3×3 kernels, on the matrix cores."""
    if not wino_eligible(x, weight):
        return F.conv2d(x, weight, bias, padding=1)
    return _WinogradConv.apply(x, weight, bias, cache or _TransformCache())


class WinogradConv2d(nn.Conv2d):
    """``nn.Conv2d`` whose 3×3 stride-1 pad-1 fp32 GPU path is the HIP Winograd kernel."""

    def __init__(self, *args, **kwargs) -> None:  # type: ignore[no-untyped-def]
        super().__init__(*args, **kwargs)
        self._wino = _TransformCache()

    def forward(self, input: Tensor) -> Tensor:
        if self.padding_mode == 'zeros' and wino_eligible(input, self.weight, self.stride,
                                                          self.padding, self.dilation,
                                                          self.groups):
            return _WinogradConv.apply(input, self.weight, self.bias, self._wino)
        # few-channel convolutions (U-Net's 3-channel input) on the implicit-GEMM kernel:
        # no MIOpen kernel to compile on the first step
        from torchgpipe_amd.ops.convbn import gemm_conv2d, gemm_conv_eligible
        if WINOGRAD_ENABLED and self.weight.shape[1] < MIN_CHANNELS and \
                gemm_conv_eligible(input, self):
            return gemm_conv2d(input, self)
        return super().forward(input)

    def __getstate__(self):  # type: ignore[no-untyped-def]
        state = self.__dict__.copy()
        state['_wino'] = _TransformCache()  # never serialise device caches
        return state
