"""Ordered running statistics for BatchNorms whose micro-batches run on several streams.

A training-mode BatchNorm folds every micro-batch's batch statistics into its running
mean / variance (``r = (1 - m) r + m x``) and counts it in ``num_batches_tracked`` -- a
read-modify-write of shared buffers, so the reference runs a stateful partition's
micro-batches strictly in order on one stream (``/root/reference/torchgpipe/pipeline.py``
``compute``; recomputations update the statistics a second time, in backward order,
``/root/reference/torchgpipe/checkpoint.py`` ``Recompute``).  Two lanes updating the same
buffers concurrently would lose updates.

:class:`OrderedRunningStats` lets the engine overlap them anyway.  Each update -- one
micro-batch's forward or recomputation through the partition -- gets a row of a per-step
slot buffer: for its duration every BatchNorm's ``running_mean`` / ``running_var`` /
``num_batches_tracked`` are that row's slices and its momentum is 1, so whichever kernel
runs (the native fused ones, MIOpen, ATen) stores the batch statistics themselves
(``0 * slot + 1 * x``) and nothing shared is touched.  :meth:`commit` then folds the rows
into the real buffers in the order the updates were *issued* -- the reference's sequential
order -- in closed form, ``r_K = (1 - m)^K r_0 + sum_k m (1 - m)^(K-1-k) x_k``, for all
BatchNorms at once on the device: a few dozen launches per step, no host sync.
"""
import contextlib
from typing import Any, Dict, Iterator, List, Optional, Tuple

import torch
from torch import Tensor, nn

__all__ = ['OrderedRunningStats']


def _tracked(module: nn.Module) -> List[nn.modules.batchnorm._BatchNorm]:
    return [m for m in module.modules()
            if isinstance(m, nn.modules.batchnorm._BatchNorm) and m.track_running_stats]


class OrderedRunningStats:
    """Per-step slots for the running statistics of ``module``'s BatchNorms (see the module
    docstring).  Use :meth:`for_module`: ``None`` when some BatchNorm cannot be slotted."""

    def __init__(self, bns: List[nn.modules.batchnorm._BatchNorm]) -> None:
        self.bns = bns
        self.sizes = [int(bn.num_features) for bn in bns]
        self.offsets: List[int] = []
        total = 0
        for c in self.sizes:
            self.offsets.append(total)
            total += c
        self.total = total
        self._mean: Optional[Tensor] = None   # [capacity, total]
        self._var: Optional[Tensor] = None
        self._count: Optional[Tensor] = None  # [capacity, len(bns)] int64
        self.used = 0
        self.live: List[int] = []  # the BatchNorms slotted this step (training mode)
        self._views: Dict[Any, Any] = {}  # row -> per-BatchNorm slices; 'live' -> the set
        self._dicts: List[Dict[str, Optional[Tensor]]] = []
        self._mods: List[nn.Module] = []
        self._orig: List[Tuple[Any, Any, Any, Any]] = []

    @staticmethod
    def for_module(module: nn.Module) -> Optional['OrderedRunningStats']:
        """Slots for every running-statistics BatchNorm of ``module``, or ``None`` when it
        has none or one of them is not a plain exponential average (a
        :class:`~torchgpipe_amd.batchnorm.DeferredBatchNorm`, which accumulates over the
        mini-batch itself; ``momentum=None``, whose factor depends on the count)."""
        from torchgpipe_amd.batchnorm import DeferredBatchNorm
        bns = _tracked(module)
        if not bns:
            return None
        for bn in bns:
            if isinstance(bn, DeferredBatchNorm) or bn.momentum is None or \
                    bn.running_mean is None or bn.running_var is None or \
                    bn.num_batches_tracked is None:
                return None
        return OrderedRunningStats(bns)

    @property
    def active(self) -> bool:
        return self._mean is not None

    def begin(self, capacity: int) -> None:
        """Open a step of at most ``capacity`` updates (a pending one is committed first).
        Only BatchNorms in training mode are slotted (an eval-mode one normalises with its
        running statistics and updates nothing); with none, the step stays inactive."""
        if self.active:
            self.commit()
        live = tuple(b for b, bn in enumerate(self.bns) if bn.training)
        self.live = list(live)
        if not live:
            return
        ref = self.bns[0].running_mean
        if self._buf_mean is None or self._buf_mean.shape[0] < capacity or \
                self._buf_mean.device != ref.device:
            self._buf_mean = torch.zeros(capacity, self.total, device=ref.device,
                                         dtype=ref.dtype)
            self._buf_var = torch.zeros_like(self._buf_mean)
            self._buf_count = torch.zeros(capacity, len(self.bns), device=ref.device,
                                          dtype=torch.long)
            self._views = {}
        else:
            self._buf_count[:capacity].zero_()
        if self._views.get('live') != live:
            self._views = {'live': live}
        self._mean, self._var, self._count = self._buf_mean, self._buf_var, self._buf_count
        self.used = 0
        # the real buffers and momenta, put back after every update
        self._dicts = [self.bns[b]._buffers for b in live]
        self._mods = [self.bns[b] for b in live]
        self._orig = [(d['running_mean'], d['running_var'], d['num_batches_tracked'],
                       m.momentum) for d, m in zip(self._dicts, self._mods)]

    _buf_mean: Optional[Tensor] = None
    _buf_var: Optional[Tensor] = None
    _buf_count: Optional[Tensor] = None

    def _row(self, k: int) -> List[Tuple[Tensor, Tensor, Tensor]]:
        """Row ``k``'s slices per live BatchNorm, made once per slot buffer (slicing ~10^4
        views per step on the host cost more than the lanes gained on ResNet p4)."""
        views = self._views.get(k)
        if views is None:
            assert self._buf_mean is not None and self._buf_var is not None and \
                self._buf_count is not None
            rm, rv, rc = self._buf_mean[k], self._buf_var[k], self._buf_count[k]
            views = [(rm[self.offsets[b]:self.offsets[b] + self.sizes[b]],
                      rv[self.offsets[b]:self.offsets[b] + self.sizes[b]], rc[b])
                     for b in self.live]
            self._views[k] = views
        return views

    @contextlib.contextmanager
    def update(self) -> Iterator[None]:
        """One update (a micro-batch's forward or recomputation through the module): the
        BatchNorms write their batch statistics into the next row instead of their
        buffers.  Host-side only, so cheap: the buffers are swapped in the modules'
        ``_buffers`` dicts (no ``nn.Module.__setattr__``) and restored on exit."""
        if not self.active:
            yield
            return
        assert self._mean is not None
        k = self.used
        if k >= self._mean.shape[0]:
            raise RuntimeError(f'more running-statistics updates than the {k} slots opened')
        self.used = k + 1
        for d, m, (rm, rv, c) in zip(self._dicts, self._mods, self._row(k)):
            d['running_mean'] = rm
            d['running_var'] = rv
            d['num_batches_tracked'] = c
            m.__dict__['momentum'] = 1.0
        try:
            yield
        finally:
            for d, m, (rm, rv, c, mom) in zip(self._dicts, self._mods, self._orig):
                d['running_mean'] = rm
                d['running_var'] = rv
                d['num_batches_tracked'] = c
                m.__dict__['momentum'] = mom

    def commit(self) -> None:
        """Fold the step's updates, in issue order, into the BatchNorms' own buffers (on the
        current stream: every stream that ran an update must have been joined to it).

        An update that did not reach a BatchNorm (its count stays 0) is skipped for it: per
        BatchNorm b and update j, the weight is ``c[j, b] m_b (1 - m_b)^(later updates of
        b)``, computed on the device -- no host sync."""
        if not self.active:
            return
        assert self._mean is not None and self._var is not None and self._count is not None
        k = self.used
        mean, var, count = self._mean[:k], self._var[:k], self._count[:k]
        self._mean = self._var = self._count = None
        self.used = 0
        if k == 0:
            return
        dev, dtype = mean.device, mean.dtype
        if self._col_bn is None or self._col_bn.device != dev:
            self._col_bn = torch.repeat_interleave(
                torch.arange(len(self.bns), device=dev),
                torch.tensor(self.sizes, device=dev))
        moms = tuple(float(bn.momentum) for bn in self.bns)  # type: ignore[arg-type]
        if self._mom is None or self._mom[0] != moms or self._mom[1].device != dev:
            # (built once: a host-to-device copy per step would wait for the stream)
            self._mom = (moms, torch.tensor(moms, dtype=torch.float64, device=dev))
        mom = self._mom[1]
        with torch.no_grad():
            c = count.to(torch.float64)                       # [k, nbn] 0 / 1
            later = c.flip(0).cumsum(0).flip(0) - c           # updates of b after j
            keep = 1.0 - mom
            w = c * mom * torch.pow(keep, later)              # [k, nbn]
            decay = torch.pow(keep, c.sum(0))                 # [nbn]
            w_col = w.index_select(1, self._col_bn).to(dtype)           # [k, total]
            decay_col = decay.index_select(0, self._col_bn).to(dtype)   # [total]
            for rows, attr in ((mean, 'running_mean'), (var, 'running_var')):
                bufs = [getattr(bn, attr) for bn in self.bns]
                new = torch.cat(bufs).mul_(decay_col).add_((w_col * rows).sum(0))
                torch._foreach_copy_(bufs, list(new.split(self.sizes)))
            torch._foreach_add_([bn.num_batches_tracked for bn in self.bns],  # type: ignore
                                list(count.sum(0).unbind()))

    _col_bn: Optional[Tensor] = None
    _mom: Optional[Tuple[Tuple[float, ...], Tensor]] = None
