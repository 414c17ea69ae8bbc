"""One pipeline stage of a multi-rank run, emulated on one device through the real engine.

:class:`LoopbackP2P` stands in for :class:`~torchgpipe_amd.parallel.p2p.P2P` so that a
:class:`~torchgpipe_amd.parallel.PipelineStage` can run as rank ``k`` of an ``n``-stage
pipeline in a single process: every receive returns pre-computed tensors of the right
shapes at once (the boundary activations and skips the preceding stages produce, or
random output gradients) and every send is dropped after its shapes are noted.  The stage
then executes exactly what it would on a multi-GPU node -- lanes, multi-stream cells,
captured cells (``graph_cells``), the fused ops' gradient accumulation, the optimizer --
minus the waits on its neighbours, so its host and device time per step are the
pipeline's per-stage costs with zero transfer time (``benchmarks/stage_harness.py``).

Receive buffers are made once per message key and reused (as ``P2P``'s persistent
receives are), so captured cells replay on them in place.
"""
from typing import Dict, Hashable, List, Optional, Sequence, Tuple

import torch
from torch import Tensor

from torchgpipe_amd.parallel.p2p import Message, TensorMeta

__all__ = ['LoopbackP2P']


class LoopbackP2P:
    """Receive pre-made tensors, drop sends (the ``P2P`` interface ``PipelineStage`` uses).

    Args:
        device: the stage's device.
        acts: the stage's input activations (one micro-batch; ignored on stage 0).
        acts_atomic: whether the activation message is a single tensor.
        skips: per source stage, the skip tensors this stage pops from it, in the stage's
            canonical route order.
        sizes: the batch size of each micro-batch when they differ (a mini-batch that does
            not split evenly: the last micro-batch is smaller); the templates are trimmed
            to it along dim 0.
    """

    stage_host = False

    def __init__(self, device: torch.device, acts: Sequence[Tensor], acts_atomic: bool,
                 skips: Dict[int, List[Tensor]],
                 sizes: Optional[Sequence[int]] = None) -> None:
        self.device = device
        self.sizes = list(sizes) if sizes is not None else None
        self.acts = [t.detach() for t in acts]
        self.acts_atomic = acts_atomic
        self.skips = {src: [t.detach() for t in ts] for src, ts in skips.items()}
        self.timeout = None
        self._sent: Dict[Hashable, List[TensorMeta]] = {}
        self._bufs: Dict[Hashable, List[Tensor]] = {}

    @staticmethod
    def _fields(key: Hashable) -> Tuple[str, int, int, int]:
        # PipelineStage._key: (signature, training, grad enabled, kind, i, src, dst)
        kind, i, src, dst = key[3:7]  # type: ignore[index]
        return kind, i, src, dst

    def send(self, tensors: Sequence[Tensor], dst: int, key: Hashable,
             atomic: bool = False, cache: bool = True) -> None:
        kind, i, src, _ = self._fields(key)
        self._sent[(kind, i, dst)] = [TensorMeta.of(t) for t in tensors]

    def _source(self, kind: str, i: int, src: int, me: int) -> List[Tuple[Tensor, bool]]:
        """(template tensor, requires_grad) of every tensor of the message."""
        if kind in ('act', 'skip'):
            ts = self.acts if kind == 'act' else self.skips.get(src, [])
            if self.sizes is not None and i < len(self.sizes):
                ts = [t[:self.sizes[i]] if t.dim() else t for t in ts]
            return [(t, t.is_floating_point()) for t in ts]
        # gradients of what this stage sent to ``src`` for micro-batch i
        # (activation gradients: only for tensors that require grad; skip gradients: one
        # per skip, zeros where none flows -- PipelineStage._backward_cells)
        sent = self._sent.get(({'gact': 'act', 'gskip': 'skip'}[kind], i, src), [])
        return [(torch.empty(m.shape, dtype=m.dtype, device=self.device), False)
                for m in sent if m.requires_grad or kind == 'gskip']

    def recv(self, src: int, key: Hashable, cache: bool = True,
             persistent: bool = False) -> Message:
        kind, i, s, me = self._fields(key)
        tmpl = self._source(kind, i, src, me)
        metas = [TensorMeta(tuple(t.shape), t.dtype, g) for t, g in tmpl]
        atomic = self.acts_atomic if kind == 'act' else False
        # buffers are made once per key (eager steps too: a fresh random tensor per receive
        # would add kernels a real stage does not run)
        bufs = self._bufs.get(key)
        if bufs is None:
            bufs = []
            for t, _ in tmpl:
                if kind in ('gact', 'gskip'):
                    b = torch.randn(t.shape, dtype=t.dtype, device=self.device) * 1e-3
                else:
                    b = t.to(self.device).clone()
                bufs.append(b)
            self._bufs[key] = bufs
        return Message([], list(bufs), None, metas, atomic)

    def send_control(self, payload: Tensor, dst: int) -> None:
        pass

    def recv_control(self, payload: Tensor, src: int) -> Tensor:
        raise RuntimeError('a loopback stage needs the step signature passed in')

    def known(self, key: Hashable) -> Optional[Tuple[List[TensorMeta], bool]]:
        return None

    def forget(self) -> None:
        self._bufs.clear()

    def flush(self) -> None:
        pass
