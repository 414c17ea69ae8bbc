"""Multi-process GPipe: one process per GPU, RCCL point-to-point between stages.

This is the MI355X-native counterpart of the reference's ``DistributedGPipe``
(``torchgpipe/distributed/gpipe.py:75-194``), re-designed around
``torch.distributed`` (RCCL over xGMI) instead of RPC with CPU staging, and
without its feature gaps: activation checkpointing with *pre-gradient*
recomputation, deferred BatchNorm and ``@skippable`` long skips all work
across processes.

Per rank ``j`` (owning partition ``j``), one training step is the GPipe
fill-drain schedule over ``m`` micro-batches::

    forward  i = 0 .. m-1:   recv act(i) from j-1, recv skips(i) from their stash ranks
                             run partition (checkpointed if i < checkpoint_stop)
                             isend act(i) to j+1, isend skips(i) to their pop ranks
    backward i = m-1 .. 0:   post recv grad(i) from j+1 and from the skip pop ranks
                             recompute(i) if checkpointed      ← overlaps the transfer
                             wait; autograd.backward(outputs(i), grads(i))
                             isend input grads to j-1 and to the skip stash ranks

Skip tensors travel directly from the stash rank to the pop rank (one xGMI
hop on the fully connected MI355X mesh), exactly like ``PortalCopy`` in the
single-process engine.

Every cell is a function ``flat_inputs → flat_outputs`` where ``flat_inputs``
= activation tensors + skips popped from other ranks and ``flat_outputs`` =
output tensors + skips stashed for other ranks, so checkpointing
(``Checkpointing``) treats cross-rank skips like any other input/output.
"""
from collections import OrderedDict
import contextlib
import datetime
import threading
import time
from typing import (Any, Callable, Dict, FrozenSet, Hashable, List, Optional, Sequence, Tuple,
                    Union)

import torch
from torch import Tensor, nn
import torch.distributed as dist

from torchgpipe_amd import microbatch
from torchgpipe_amd.batchnorm import DeferredBatchNorm, set_micro_batches
from torchgpipe_amd.checkpoint import Checkpointing
from torchgpipe_amd.gpipe import check_balance, partition_layers, verify_module
from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.ops.conv import new_step as wino_new_step
from torchgpipe_amd.ops.conv import hold_cache, refresh_step_caches, size_cache_budget
from torchgpipe_amd.ops.dropout import convert_dropout
from torchgpipe_amd.ops.fusion import relink
from torchgpipe_amd.parallel.p2p import _DTYPE_CODE, P2P, _wait
from torchgpipe_amd.runstats import OrderedRunningStats
from torchgpipe_amd.skip.layout import SkipLayout, inspect_skip_layout
from torchgpipe_amd.skip.namespace import Namespace
from torchgpipe_amd.skip.skippable import Skippable, verify_skippables
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker
from torchgpipe_amd.stream import named_stream
from torchgpipe_amd.utils import trace
from torchgpipe_amd.utils.meta import is_meta
from torchgpipe_amd.utils.meta import materialize as meta_materialize

__all__ = ['PipelineStage', 'signature_of', 'stream_census', 'link_pairs', 'HW_QUEUES']

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]
Key = Tuple[Namespace, str]
Signature = Tuple[Any, ...]


def signature_of(input: TensorOrTensors) -> Signature:
    """Hashable description of a mini-batch: shape and dtype code of each tensor."""
    tensors = (input,) if isinstance(input, Tensor) else tuple(input)
    return tuple((tuple(t.shape), _DTYPE_CODE[t.dtype]) for t in tensors)


def _encode_signature(sig: Signature) -> Tensor:
    words: List[int] = [len(sig)]
    for shape, code in sig:
        words += [len(shape), *shape, code]
    out = torch.zeros(128, dtype=torch.int64)
    out[:len(words)] = torch.tensor(words, dtype=torch.int64)
    return out


def _decode_signature(payload: Tensor) -> Signature:
    words = payload.tolist()
    count, pos = words[0], 1
    sig = []
    for _ in range(count):
        ndim = words[pos]
        shape = tuple(words[pos + 1:pos + 1 + ndim])
        sig.append((shape, words[pos + 1 + ndim]))
        pos += 2 + ndim
    return tuple(sig)


def _micro_batch_count(sig: Signature, chunks: int) -> int:
    batch = sig[0][0][0] if sig and sig[0][0] else 1
    return len(torch.empty(batch, 0).chunk(chunks)) if batch > 0 else 0


@contextlib.contextmanager
def _shared_accumulators() -> Any:
    """Backward passes of micro-batches that ran on different lanes.

    A parameter whose gradient autograd accumulates (one the fused ops do not write into
    ``.grad`` themselves: MIOpen strided convolutions, Linear layers) has one
    ``AccumulateGrad`` node per step, shared by the graphs of every micro-batch alive at
    once and bound to the stream of the micro-batch that created it.  Lanes put those
    micro-batches on different streams by design, so the engine orders each accumulation
    after the producing lane (the ordering the lanes need) and warns about the mismatch;
    here it is intentional, and the warning is off for the duration of the backward.

    The flag is process-global: nested or concurrent stages count their holders, and the
    last one out restores what the flag was before the first one came in (a user's own
    ``set_warn_on_accumulate_grad_stream_mismatch(False)`` stays in force).
    """
    global _accumulator_holders, _accumulator_saved
    with _accumulator_lock:
        if _accumulator_holders == 0:
            _accumulator_saved = bool(torch._C._warn_on_accumulate_grad_stream_mismatch())
            torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(False)
        _accumulator_holders += 1
    try:
        yield
    finally:
        with _accumulator_lock:
            _accumulator_holders -= 1
            if _accumulator_holders == 0:
                torch.autograd.graph.set_warn_on_accumulate_grad_stream_mismatch(
                    _accumulator_saved)


_accumulator_lock = threading.Lock()
_accumulator_holders = 0
_accumulator_saved = True


def _loss_leaves(loss: Tensor, outputs: Sequence[Tensor]) -> List[Tensor]:
    """The leaves (e.g. a loss head's parameters) whose gradient ``loss`` reaches without
    passing through ``outputs``: the last stage's direct backward stops at the outputs,
    so these need their own share of the pass.  Walks the loss's graph up to the
    outputs' nodes (a few nodes for the usual loss functions)."""
    stop = {t.grad_fn for t in outputs if t.grad_fn is not None}
    leaves: List[Tensor] = []
    seen = set()
    todo = [loss.grad_fn]
    while todo:
        node = todo.pop()
        if node is None or node in seen or node in stop:
            continue
        seen.add(node)
        var = getattr(node, 'variable', None)
        if var is not None and var.requires_grad:
            leaves.append(var)
            continue
        todo.extend(nxt for nxt, _ in node.next_functions)
    return leaves


class _RemoteSkipTracker(SkipTracker):
    """Skip tracker of one cell: local skips in a dict, cross-rank ones captured."""

    def __init__(self, layout: SkipLayout, rank: int, popped: Dict[Key, Tensor]) -> None:
        super().__init__()
        self.layout = layout
        self.rank = rank
        self.popped = popped
        self.stashed: Dict[Key, Optional[Tensor]] = {}

    def save(self, batch: Batch, ns: Namespace, name: str, tensor: Optional[Tensor]) -> None:
        src, dst = self.layout.route(ns, name)
        if dst != self.rank:
            self.stashed[(ns, name)] = tensor
        else:
            super().save(batch, ns, name, tensor)

    def load(self, batch: Batch, ns: Namespace, name: str) -> Optional[Tensor]:
        src, dst = self.layout.route(ns, name)
        if src != self.rank:
            return self.popped.pop((ns, name))
        return super().load(batch, ns, name)


class _Cell:
    """Bookkeeping of one micro-batch on this rank."""

    __slots__ = ('index', 'inputs', 'outputs', 'out_atomic', 'chk', 'n_act_out', 'lane', 'fn',
                 'seg')

    def __init__(self, index: int) -> None:
        self.index = index
        self.fn: Optional[Callable[[Tensors], Tensors]] = None  # (segments: for the capture)
        self.seg = False  # a captured cell (parallel/segments.py)
        self.inputs: List[Tensor] = []      # leaves: activations + popped remote skips
        self.outputs: List[Tensor] = []     # outputs + stashed remote skips
        self.out_atomic = True
        self.chk: Optional[Checkpointing] = None
        self.n_act_out = 0
        self.lane: Optional[torch.cuda.Stream] = None  # stream it was recomputed on


def link_pairs(layout: SkipLayout, n: int) -> List[Tuple[int, int]]:
    """Stage pairs of an ``n``-stage pipeline that exchange messages: neighbours plus the
    cross-stage skip routes of ``layout`` (each pair: one link, one RCCL communicator)."""
    pairs = {(j, j + 1) for j in range(n - 1)}
    for (src, dst) in layout.by_ns_name.values():
        if src != dst:
            pairs.add((min(src, dst), max(src, dst)))
    return sorted(pairs)


# GPU_MAX_HW_QUEUES that bench.py sets for multi-rank runs (the most the runtime is given
# on this pool).  A rank's own streams and its RCCL communicators' streams must fit with
# room to spare -- CENSUS_LIMIT, for the default stream and library streams -- or a spinning
# receive shares a hardware queue with (and blocks) unrelated work
# (tests/test_stream_census.py).
HW_QUEUES = 32
CENSUS_LIMIT = 24


def stream_census(rank: int, pairs: Sequence[Tuple[int, int]], *, forward_lanes: bool,
                  recompute_lanes: bool, cell_streams: int = 0, graph_cells: bool = False,
                  relay_routes: int = 0, relay_links: int = 0) -> Dict[str, int]:
    """Streams a pipeline rank queues work on: the compute stream, two forward lanes, two
    recompute lanes, an AmoebaNet cell's side streams (``cell_streams - 1``), the captured
    cells' two streams, one stream per relayed route (``parallel/p2p.py`` begin_relays),
    and one RCCL communicator stream per link and per relay link it is part of."""
    links = sum(1 for a, b in pairs if rank in (a, b))
    out = {'compute': 1, 'forward_lanes': 2 if forward_lanes else 0,
           'recompute_lanes': 2 if recompute_lanes else 0,
           'cell_side_streams': max(0, cell_streams - 1), 'graph_cells': 2 if graph_cells else 0,
           'relay_routes': relay_routes, 'link_comms': links, 'relay_comms': relay_links}
    out['total'] = sum(out.values())
    return out


# 2-rank relay communicators of multi-path transfers, per WORLD group, per GPU pair
_RELAY_LINKS: Dict[int, Dict[FrozenSet[int], Any]] = {}


class PipelineStage:
    """One pipeline stage of a multi-process GPipe (this rank's partition).

    Args:
        module: the *whole* ``nn.Sequential`` (it may live on the ``meta``
            device; only this rank's layers are materialised).
        balance: layers per partition; ``len(balance)`` = pipeline depth.
        rank: this rank's stage index (default: rank in ``group``).
        device: device of this stage (default: ``cuda:LOCAL_RANK`` or CPU).
        chunks: number of micro-batches.
        checkpoint: ``'always'``, ``'except_last'`` or ``'never'``.
        group: process group of the pipeline (default: WORLD); its size must
            equal ``len(balance)``.
        ctrl_group: ``gloo`` group for shape metadata (default: WORLD if it is
            gloo, otherwise a new gloo group over the same ranks).
        deferred_batch_norm: convert BatchNorm layers to DeferredBatchNorm.
        philox_dropout: ``nn.Dropout`` / ``nn.Dropout2d`` on tape-replayed Philox pairs
            (``ops.dropout.convert_dropout``), as for ``GPipe``.
        pack: pack multi-tensor messages into one transfer (HIP kernel).
        links: one 2-rank communicator per used link (default: on for RCCL,
            off for gloo).
        materialize: called on this rank's partition before it is moved to
            ``device`` (e.g. to initialise layers built on the ``meta`` device).
        graph_cells: replay every checkpointed micro-batch's forward, recomputation and
            backward as captured hipGraphs, with the transfers issued eagerly in between
            (``parallel/segments.py``): after ``graph_warmup`` eager steps and one capture
            step, the host launches three graphs per cell instead of every kernel.  GPU
            stages only; gradients accumulate across steps as in eager mode (the captured
            backward adds into ``.grad``, which is zeroed only where the user released it:
            ``parallel/segments.py``).
        graph_warmup: eager steps before the capture step (the first runs without cached
            weight transforms and sizes their budget, the second fills the caches, so the
            capture reads them instead of recomputing transforms in its graphs).
        transport: a stand-in for the point-to-point layer (``P2P`` interface), e.g.
            :class:`~torchgpipe_amd.parallel.loopback.LoopbackP2P` to run this stage as
            ``rank`` of a ``len(balance)``-stage pipeline in one process without
            ``torch.distributed`` (single-device stage emulation); ``rank`` is required.
        timeout: seconds any host-blocking wait of this stage (shape metadata,
            control messages, gloo tensors) may take before raising
            :class:`~torchgpipe_amd.parallel.p2p.PipelineTimeout`; also the
            timeout of the groups this stage creates.  ``None`` = the default
            group's timeout.  RCCL transfers are bounded by the RCCL process
            group's own watchdog timeout (``init_process_group(timeout=...)``).
        stripes: multi-path transfers (``parallel/stripes.py``): messages of at least this
            many bytes on a route that carries one kind of message also travel through up
            to ``stripe_relays`` idle ranks, over links no pipeline traffic uses.  Planned
            from the first training step of each step signature (recorded) at the start
            of the second (collective on the control group); ``None`` = off.  Needs a
            third rank and the pipeline group spanning WORLD (relay links are created with
            ``new_group``); otherwise a no-op.
        stripe_relays: the most relays one route takes.
        direct_backward: back-propagate a recomputed micro-batch straight through its
            recomputed graph (one autograd engine call) instead of through its Checkpoint
            node, whose backward re-enters the engine for the same work (default on; off
            restores the reference's Checkpoint/Recompute choreography exactly).
        backward_thread: issue each micro-batch's backward from a helper thread, so the
            host enqueues the next micro-batch's recomputation (and posts its receives)
            while the autograd engine enqueues this backward: the two host streams of
            kernel launches overlap where they release the GIL.  Measured on the
            launch-bound stages (AmoebaNet and ResNet-101 at 22-40-image micro-batches):
            no gain, the host time is GIL-held Python (profiles/r5/backward_thread.md);
            off by default.  Eager cells only.
    """

    def __init__(self, module: nn.Sequential, balance: Sequence[int], *,
                 rank: Optional[int] = None, device: Optional[torch.device] = None,
                 chunks: int = 1, checkpoint: str = 'except_last',
                 group: Optional[dist.ProcessGroup] = None,
                 ctrl_group: Optional[dist.ProcessGroup] = None,
                 deferred_batch_norm: bool = False, pack: bool = True,
                 links: Optional[bool] = None,
                 materialize: Optional[Callable[[nn.Module], None]] = None,
                 timeout: Optional[float] = None,
                 overlap_recompute: bool = False,
                 overlap_forward: bool = False,
                 philox_dropout: bool = False,
                 graph_cells: bool = False,
                 graph_warmup: int = 2,
                 transport: Optional[Any] = None,
                 stripes: Optional[int] = None,
                 stripe_relays: int = 3,
                 backward_thread: bool = False,
                 direct_backward: bool = True) -> None:
        if chunks <= 0:
            raise ValueError('number of chunks must be positive integer')
        if checkpoint not in ('always', 'except_last', 'never'):
            raise ValueError("checkpoint is not one of 'always', 'except_last', or 'never'")
        verify_module(module)
        verify_skippables(module)
        balance = list(balance)
        check_balance(module, balance)

        self.group = group
        distributed = dist.is_available() and dist.is_initialized() and transport is None
        if transport is not None:
            if rank is None:
                raise ValueError('a stage on a stand-in transport needs its rank')
            self.world, self.rank = len(balance), rank
        else:
            if not distributed and len(balance) != 1:
                raise RuntimeError('a multi-stage pipeline needs torch.distributed to be '
                                   'initialized')
            self.world = dist.get_world_size(group) if distributed else 1
            self.rank = (dist.get_rank(group) if distributed else 0) if rank is None else rank
        if self.world != len(balance):
            raise ValueError(f'pipeline group has {self.world} ranks but balance has '
                             f'{len(balance)} partitions')
        self.ranks = [dist.get_global_rank(group, r) if group is not None and distributed
                      else r for r in range(self.world)]
        self.n = len(balance)
        self.balance = balance
        self.chunks = chunks
        self.checkpoint = checkpoint
        self.training = True
        self.timeout = timeout
        group_kwargs: Dict[str, Any] = ({} if timeout is None else
                                        {'timeout': datetime.timedelta(seconds=timeout)})

        if device is None:
            device = torch.device('cpu')
        self.device = device

        groups = partition_layers(module, balance)
        parts = [nn.Sequential(g) for g in groups]
        # every partition's layer names (checkpoint index: which shard holds which layers)
        self.layer_names = [[name for name, _ in part.named_children()] for part in parts]
        self.layout = inspect_skip_layout(parts)
        partition = parts[self.rank]
        if deferred_batch_norm:
            partition = DeferredBatchNorm.convert_deferred_batch_norm(partition, chunks)
        if philox_dropout:  # user dropout layers on the checkpoint's RNG tape
            convert_dropout(partition)
        if materialize is not None:
            materialize(partition)
        if is_meta(partition):
            # Whole model built on the meta device: only this rank's layers get memory.
            meta_materialize(partition, device)
        self.partition = partition.to(device)
        # Conv-BN(-ReLU) runs fuse only inside this partition (ops/fusion.py)
        relink(self.partition)
        self._has_dbn = any(isinstance(m, DeferredBatchNorm) for m in partition.modules())

        # Cross-rank skip routes touching this rank, in a canonical order that every
        # rank derives identically: (peer, global index of the stash layer, name).
        # Namespaces are random UUIDs that differ between processes, so they
        # must never decide the order.
        stash_index: Dict[Key, int] = {}
        for idx, layer in enumerate(module.children()):
            if isinstance(layer, Skippable):
                for key in layer.stashable():
                    stash_index[key] = idx
        self.in_skips: List[Tuple[int, Key]] = sorted(
            ((src, (ns, name)) for src, ns, name in self.layout.copy_policy(self.rank)),
            key=lambda r: (r[0], stash_index[r[1]], r[1][1]))
        self.out_skips: List[Tuple[int, Key]] = sorted(
            ((dst, (ns, name)) for dst, ns, name in self.layout.send_policy(self.rank)),
            key=lambda r: (r[0], stash_index[r[1]], r[1][1]))

        if ctrl_group is None and distributed:
            if dist.get_backend(group) == 'gloo':
                ctrl_group = group
            else:
                ctrl_group = dist.new_group(ranks=self.ranks, backend='gloo', **group_kwargs)
        self.ctrl_group = ctrl_group
        self.p2p = transport if transport is not None else \
            P2P(device, group=group, ctrl_group=ctrl_group, pack=pack,
                link_groups=self._make_links(links, group_kwargs) if distributed else None,
                timeout=timeout)

        self._cells: List[_Cell] = []
        self.overlap_recompute = overlap_recompute
        self.overlap_forward = overlap_forward
        self._lanes: Optional[List[torch.cuda.Stream]] = None
        self._fwd_lanes: Optional[List[torch.cuda.Stream]] = None
        # modules whose forward carries state across micro-batches (running statistics):
        # their micro-batches must run in order on one stream
        self._stateful = any(isinstance(m, nn.modules.batchnorm._BatchNorm)
                             and m.track_running_stats for m in self.partition.modules())
        # ... unless their running statistics can be slotted per update and folded in order
        # (runstats.py): then their forwards and recomputations may overlap on lanes too
        self._stat_slots: Optional[OrderedRunningStats] = \
            OrderedRunningStats.for_module(self.partition) if self._stateful else None
        self._rec_slotted = False  # this step's recomputations are slotted
        self._sig: Optional[Signature] = None
        self._m = 0
        self._probe: Optional[List[Tuple[str, Any, Any]]] = None
        if graph_warmup < 1:
            raise ValueError('graph_cells needs at least one eager warm-up step')
        self.graph_cells = graph_cells and device.type == 'cuda'
        if graph_cells:
            from torchgpipe_amd.batchnorm import DeferredBatchNorm as _DBN
            if any(isinstance(m, _DBN) and m.momentum is None
                   for m in self.partition.modules()):
                # the cumulative average's factor 1/n is read on the host at commit time:
                # a captured commit would freeze it
                raise ValueError('graph_cells does not support DeferredBatchNorm with '
                                 'momentum=None (cumulative moving average)')
        self.graph_warmup = graph_warmup
        self._segments: Optional[Any] = None
        self._seg_key: Optional[Tuple[Any, ...]] = None
        self._seg_phase = 'eager'
        self._persistent = False  # this step receives into persistent buffers
        # derived-weight cache budget: None = not sized yet, 'measuring' = first step ran
        # uncached (ops/conv.py size_cache_budget), 'sized'
        self._cache_state: Optional[str] = None
        # multi-path transfers: per step signature 'record' (first training step records
        # its sends), the recorded sends, then the plan
        whole = distributed and self.n == dist.get_world_size()
        self._stripe_min = int(stripes or 0) if whole and self.n > 2 else 0
        self._stripe_relays = stripe_relays
        self._stripe_plans: Dict[Any, Any] = {}
        self._stripe_on = False  # this step runs a plan (or records)
        self._stripe_sig: Optional[Signature] = None
        self._group_kwargs = group_kwargs
        self.backward_thread = backward_thread
        self.direct_backward = direct_backward
        self._bwd_pool: Optional[Any] = None
        if distributed and self.n > 1:
            self.connect()

    def _segments_for(self, sig: Signature, stop: int) -> Optional[Any]:
        """The captured cells for this step's signature (``None``: eager step)."""
        if not self.graph_cells or not self.training or \
                not torch.is_grad_enabled() or torch.cuda.is_current_stream_capturing():
            return None
        key = (sig, stop)
        if self._segments is None or self._seg_key != key:
            from torchgpipe_amd.parallel.segments import Segments
            self._segments = Segments(self.partition, self.device,
                                      _micro_batch_count(sig, self.chunks), stop,
                                      self.graph_warmup)
            self._seg_key = key
        return self._segments

    @property
    def graph_phase(self) -> str:
        """Phase of the last step with ``graph_cells``: 'eager', 'capture' or 'replay'."""
        return self._seg_phase

    def _link_pairs(self) -> List[Tuple[int, int]]:
        """Stage pairs that exchange messages: neighbours plus cross-rank skip routes."""
        return link_pairs(self.layout, self.n)

    def stream_census(self) -> Dict[str, int]:
        """The HIP streams this rank's engine runs work on, and the RCCL communicators
        (each with a stream of its own) it is part of: :func:`stream_census` of this
        stage's options, links and (once planned) relay routes."""
        from torchgpipe_amd.parallel.p2p import StripePlan
        plan = self._stripe_plans.get(self._sig)
        me = self.ranks[self.rank]
        jobs = len(plan.jobs) if isinstance(plan, StripePlan) else 0
        relay_links = sum(1 for k in self.p2p.relay_links if me in k) \
            if hasattr(self.p2p, 'relay_links') else 0
        cells = [getattr(m, 'streams', 0) for m in self.partition.modules()]
        return stream_census(self.rank, link_pairs(self.layout, self.n),
                             forward_lanes=self.overlap_forward and self._lanes_ok(),
                             recompute_lanes=self.overlap_recompute,
                             cell_streams=max([c for c in cells if isinstance(c, int)] + [0]),
                             graph_cells=self.graph_cells, relay_routes=jobs,
                             relay_links=relay_links)

    def connect(self) -> None:
        """Open every link this stage uses, in one global order.

        RCCL creates a peer pair's communicator on the first send/recv between
        them, and that creation blocks both hosts until the pair meets.  Left
        to the training step, the order in which a rank meets its peers follows
        its own message order (activations first, then skips), and stages with
        skips to distant ranks could wait on each other in a cycle.  Here every
        rank visits its pairs in the same sorted order, which cannot cycle, and
        exchanges one element per pair, so all communicators exist before the
        first step.
        """
        staged = self.p2p.stage_host or self.device.type != 'cuda'
        where = torch.device('cpu') if staged else self.device
        works = []
        for a, b in self._link_pairs():
            if self.rank not in (a, b):
                continue
            peer = self.ranks[b if self.rank == a else a]
            buf = torch.zeros(1, device=where)
            if self.rank == a:
                works.append(dist.isend(buf, peer, group=self.p2p._link(peer)))
            else:
                _wait(dist.irecv(buf, peer, group=self.p2p._link(peer)),
                      self.p2p.timeout if staged else None, f'link handshake with rank {peer}')
        for w in works:
            _wait(w, self.p2p.timeout if staged else None, 'link handshake')
        if where.type == 'cuda':
            torch.cuda.synchronize(where)

    def _make_links(self, enabled: Optional[bool], group_kwargs: Dict[str, Any]
                    ) -> Dict[int, dist.ProcessGroup]:
        """Create one 2-rank process group per pipeline link this model uses.

        ``new_group`` is collective over WORLD, so every rank creates every
        link in the same (sorted) order, including links it is not part of.
        Links are the adjacent-stage pairs plus every cross-partition skip route.
        On ``gloo`` (CPU) the pipeline group itself is used.
        """
        if enabled is None:
            # Needed only when the group was eagerly initialised (``device_id``):
            # then PyTorch runs unbatched P2P on the group's single communicator.
            # Lazily initialised RCCL groups already give every peer pair its own
            # communicator (and stream) on first use.
            pg = self.group if self.group is not None else dist.group.WORLD
            enabled = (dist.get_backend(self.group) != 'gloo'
                       and getattr(pg, 'bound_device_id', None) is not None)
        if not enabled:
            return {}
        links: Dict[int, dist.ProcessGroup] = {}
        for a, b in self._link_pairs():
            pg = dist.new_group(ranks=[self.ranks[a], self.ranks[b]], **group_kwargs)
            if self.rank == a:
                links[self.ranks[b]] = pg
            elif self.rank == b:
                links[self.ranks[a]] = pg
        return links

    # -- module-like helpers ----------------------------------------------------------------

    def parameters(self):  # type: ignore[no-untyped-def]
        return self.partition.parameters()

    def train(self, mode: bool = True) -> 'PipelineStage':
        self.training = mode
        self.partition.train(mode)
        return self

    def eval(self) -> 'PipelineStage':
        return self.train(False)

    @property
    def is_first(self) -> bool:
        return self.rank == 0

    @property
    def is_last(self) -> bool:
        return self.rank == self.n - 1

    def checkpoint_stop(self, m: int) -> int:
        # Like GPipe.checkpoint_stop: checkpointing only while training.
        if not (self.training and torch.is_grad_enabled()):
            return 0
        return {'always': m, 'except_last': m - 1, 'never': 0}[self.checkpoint]

    # -- signature --------------------------------------------------------------------------

    def _agree_signature(self, input: Optional[TensorOrTensors],
                         signature: Optional[Signature]) -> Signature:
        """Every rank needs the step's input signature (micro-batch count, meta keys).

        Rank 0 ships it to the others over the gloo control group (non-blocking
        sends, so rank 0 never waits for a rank still busy with the previous
        step).  Callers that know the signature on every rank pass it in and
        skip this exchange.
        """
        if signature is not None:
            return signature
        if self.is_first:
            if input is None:
                raise ValueError('the first stage needs the input mini-batch')
            sig = signature_of(input)
            payload = _encode_signature(sig)
            for r in range(1, self.n):
                self.p2p.send_control(payload, self.ranks[r])
            return sig
        payload = torch.zeros(128, dtype=torch.int64)
        self.p2p.recv_control(payload, self.ranks[0])
        return _decode_signature(payload)

    def _key(self, kind: str, i: int, src: int, dst: int) -> Hashable:
        # Metadata cache key of one message.  Both endpoints are part of it: a
        # stage may send the same kind of message (skips, skip gradients) to
        # several peers in one micro-batch, each with its own layout.
        return (self._sig, self.training, torch.is_grad_enabled(), kind, i, src, dst)

    # -- forward ----------------------------------------------------------------------------

    def _make_fn(self, cell: _Cell, n_act: int, in_atomic: bool
                 ) -> Callable[[Tensors], Tensors]:
        in_keys = [key for _, key in self.in_skips]
        out_keys = [key for _, key in self.out_skips]
        partition = self.partition
        label = f'fwd mb{cell.index} stage{self.rank}'

        def fn(flat: Tensors) -> Tensors:
            acts = flat[:n_act]
            popped = dict(zip(in_keys, flat[n_act:]))
            tracker = _RemoteSkipTracker(self.layout, self.rank, popped)
            with use_skip_tracker(tracker), trace.range(label):
                out = partition(acts[0] if in_atomic else tuple(acts))
            batch = Batch(out)
            cell.out_atomic = batch.atomic
            cell.n_act_out = len(batch)
            stashed = []
            for key in out_keys:
                t = tracker.stashed.get(key)
                if t is None:
                    raise RuntimeError(f"skip '{key[1]}' was not stashed")
                stashed.append(t)
            return tuple(batch) + tuple(stashed)

        return fn

    def forward(self, input: Optional[TensorOrTensors] = None, *,
                signature: Optional[Signature] = None) -> List[TensorOrTensors]:
        """Run the forward pass of every micro-batch on this stage.

        The first stage passes the mini-batch; the others pass ``None``.
        Returns the per-micro-batch outputs (meaningful on the last stage).
        """
        if input is not None:
            microbatch.check(input)
        wino_new_step()  # weights may have changed since the last step (even via .data)
        sig = self._agree_signature(input, signature)
        if sig != self._sig:
            self._sig = sig
        m = _micro_batch_count(sig, self.chunks)
        self._m = m
        if self._has_dbn:
            set_micro_batches(self.partition, m)
        stop = self.checkpoint_stop(m)
        if self.device.type == 'cuda':
            if self._cache_state is None and self.training and torch.is_grad_enabled():
                # the first training step runs without cached weight transforms: its peak
                # sizes the cache (at most a fraction of the stage's own footprint)
                hold_cache(self.device)
                self._cache_state = 'measuring'
            # derived weights recomputed in place, on this stream, before any lane reads them
            refresh_step_caches(self.partition)
        self._stripe_begin(sig)
        seg = self._segments_for(sig, stop)
        phase = seg.begin_step() if seg is not None else 'eager'
        self._seg_phase = phase
        graphed = phase in ('capture', 'replay')
        persistent = self._persistent = seg is not None

        batches: Optional[List[Batch]] = None
        if self.is_first:
            assert input is not None
            batches = microbatch.scatter(input, self.chunks)

        me = self.ranks[self.rank]
        prev = self.ranks[self.rank - 1] if self.rank > 0 else None
        nxt = self.ranks[self.rank + 1] if not self.is_last else None
        self._cells = []
        outputs: List[TensorOrTensors] = []

        flanes = self._forward_lanes() if not (graphed and self._stateful) else None
        main = torch.cuda.current_stream(self.device) if flanes is not None else None
        slots = self._stat_slots if self._stateful and flanes is not None else None
        if slots is not None:
            slots.begin(m)
        for i in range(m):
            cell = _Cell(i)
            # 1. inputs: activations + cross-rank skips (posted before waiting on any)
            if self.is_first:
                assert batches is not None
                b = batches[i]
                acts = [t.to(self.device, non_blocking=True) for t in b]
                in_atomic = b.atomic
                act_msg = None
            else:
                act_msg = self.p2p.recv(prev, self._key('act', i, prev, me),  # type: ignore[arg-type]
                                        persistent=persistent)
                in_atomic = True
            skip_msgs = [self.p2p.recv(self.ranks[src], self._key('skip', i, self.ranks[src], me),
                                       persistent=persistent)
                         for src in sorted({s for s, _ in self.in_skips})]
            mark = self._probe_begin() if act_msg is not None or skip_msgs else None
            if act_msg is not None:
                acts = act_msg.wait()
                in_atomic = act_msg.atomic
            popped: List[Tensor] = []
            for msg in skip_msgs:
                popped += msg.wait()
            self._probe_end('fwd', mark)
            flat = list(acts) + popped
            cell.inputs = flat

            # 2. compute (independent micro-batches of a one-rank, stateless partition
            #    alternate between two forward lanes)
            fn = self._make_fn(cell, len(acts), in_atomic)
            lane = None
            if graphed:
                # a captured cell: its graphs read the persistent inputs in place
                assert seg is not None
                sc = seg.cells[i]
                fresh = sc.fwd is None
                if fresh:
                    flat = seg.adopt_inputs(i, flat, owned=self.is_first)
                else:
                    flat = seg.static_inputs(i, flat)
                cell.inputs = flat
                cell.seg = True
                cell.fn = fn if sc.rec is None else None
                if flanes is not None:
                    lane = flanes[i % 2]
                run = lane if lane is not None else torch.cuda.current_stream(self.device)
                with trace.range(f'fwd graph mb{i} stage{self.rank}'):
                    seg.forward(i, fn, run)
                if fresh:  # the capture ran fn: it described the outputs
                    sc.out_atomic, sc.n_act_out = cell.out_atomic, cell.n_act_out
                else:
                    cell.out_atomic, cell.n_act_out = sc.out_atomic, sc.n_act_out
                out = seg.user_outputs(i)
            elif flanes is not None:
                assert main is not None
                lane = flanes[i % 2]
                lane.wait_stream(main)
                for t in flat:
                    t.record_stream(lane)
            if not cell.seg:
                with torch.cuda.stream(lane) if lane is not None else contextlib.nullcontext(), \
                        slots.update() if slots is not None else contextlib.nullcontext():
                    if i < stop:
                        cell.chk = Checkpointing(fn, Batch(tuple(flat)))
                        out = list(cell.chk.checkpoint())
                    else:
                        out = list(fn(tuple(flat)))
            if lane is not None and not cell.seg:
                assert main is not None
                for t in out:
                    t.record_stream(main)
                if cell.chk is None:
                    cell.lane = lane  # its backward runs there (ordered in _backward)
            cell.outputs = out
            self._cells.append(cell)

            # 3. outputs: activation to the next stage, skips to their pop ranks.  Sends
            #    are ordered after the stream that computed them (RCCL syncs with the
            #    current stream), so a lane's outputs leave without holding up main.
            act_out = out[:cell.n_act_out]
            with torch.cuda.stream(lane) if lane is not None else contextlib.nullcontext():
                if nxt is not None:
                    self.p2p.send(act_out, nxt, self._key('act', i, me, nxt),
                                  atomic=cell.out_atomic)
                by_dst: Dict[int, List[Tensor]] = OrderedDict()
                for (dst, _), t in zip(self.out_skips, out[cell.n_act_out:]):
                    by_dst.setdefault(dst, []).append(t)
                for dst in sorted(by_dst):
                    self.p2p.send(by_dst[dst], self.ranks[dst],
                                  self._key('skip', i, me, self.ranks[dst]))
            outputs.append(act_out[0] if cell.out_atomic else tuple(act_out))
        if flanes is not None and main is not None:
            for lane in flanes:
                main.wait_stream(lane)
        if slots is not None:
            slots.commit()  # the forwards' running-statistics updates, in micro-batch order
        if not torch.is_grad_enabled():
            # Inference: no backward will flush the sends; complete them now.
            self.p2p.flush()
            self._cells = []
        return outputs

    # -- multi-path transfers ---------------------------------------------------------------

    @property
    def stripes_ready(self) -> bool:
        """Whether the last step's signature runs its stripe plan (or striping is off)."""
        if not self._stripe_min:
            return True
        from torchgpipe_amd.parallel.p2p import StripePlan
        return isinstance(self._stripe_plans.get(self._sig), StripePlan)

    @property
    def striped_routes(self) -> Dict[str, List[int]]:
        """The last step signature's striped routes, ``'src->dst': relays`` (global ranks)."""
        from torchgpipe_amd.parallel.p2p import StripePlan
        plan = self._stripe_plans.get(self._sig)
        if not isinstance(plan, StripePlan):
            return {}
        return {f'{a}->{b}': list(r) for (a, b), r in sorted(plan.stripes.items())}

    def _stripe_begin(self, sig: Signature) -> None:
        """Start this step's multi-path transfers (``parallel/stripes.py``)."""
        if not self._stripe_min:
            return
        p2p = self.p2p
        self._stripe_end()
        if not (self.training and torch.is_grad_enabled()):
            p2p.use_plan(None)
            return
        state = self._stripe_plans.get(sig)
        if state is None or state == 'record':
            # first training step of this signature: every rank records what it sends
            self._stripe_plans[sig] = 'record'
            self._stripe_sig = sig
            p2p.use_plan(None)
            p2p.start_recording()
            self._stripe_on = True
            return
        if isinstance(state, list):  # recorded last step: plan now, on every rank alike
            state = self._stripe_plans[sig] = self._make_stripe_plan(state)
        p2p.use_plan(state)
        p2p.begin_relays()
        self._stripe_on = True

    def _stripe_end(self) -> None:
        """End the step's multi-path transfers: keep the recording, join the relays."""
        if not self._stripe_on:
            return
        self._stripe_on = False
        p2p = self.p2p
        if p2p._recording is not None:
            self._stripe_plans[self._stripe_sig] = p2p.stop_recording()
        else:
            p2p.end_relays()
        p2p.use_plan(None)

    def _make_stripe_plan(self, mine: List[Any]) -> Any:
        from torchgpipe_amd.parallel import stripes as stripes_mod
        from torchgpipe_amd.parallel.p2p import StripePlan
        me = self.ranks[self.rank]
        gathered: List[Any] = [None] * self.n
        dist.all_gather_object(gathered, (me, [tuple(s) for s in mine]),
                               group=self.ctrl_group)
        sends = {r: [stripes_mod.Send(*s) for s in lst] for r, lst in gathered}
        routes, jobs = stripes_mod.plan(sends, self.ranks, self._stripe_min,
                                        self._stripe_relays)
        sizes: Dict[Tuple[int, int], List[int]] = {}
        for src, lst in sends.items():
            for s in lst:
                if (src, s.dst) in routes and s.nbytes >= self._stripe_min:
                    sizes.setdefault((src, s.dst), []).append(s.nbytes)
        pairs = sorted({tuple(sorted((end, r))) for (src, dst), relays in routes.items()
                        for r in relays for end in (src, dst)})
        self._open_relay_links(pairs)
        return StripePlan(routes, sizes, jobs.get(me, []), self._stripe_min)

    def _open_relay_links(self, pairs: List[Tuple[int, int]]) -> None:
        """One 2-rank group per detour pair (``new_group`` is collective: every rank creates
        every pair, in one sorted order), each opened with a one-element exchange in that
        order, like :meth:`connect`."""
        links = self.p2p.relay_links
        me = self.ranks[self.rank]
        # shared by every stage of this process (bench.py builds several): every rank
        # creates the same pairs in the same order, so the cache stays in step across ranks
        shared = _RELAY_LINKS.setdefault(id(dist.group.WORLD), {})
        for a, b in pairs:
            key = frozenset((a, b))
            if key not in shared:
                shared[key] = dist.new_group(ranks=[a, b], **self._group_kwargs)
            links[key] = shared[key]
        staged = self.p2p.stage_host or self.device.type != 'cuda'
        where = torch.device('cpu') if staged else self.device
        works = []
        for a, b in pairs:
            if me not in (a, b):
                continue
            pg = links[frozenset((a, b))]
            buf = torch.zeros(1, device=where)
            if me == a:
                works.append(dist.isend(buf, b, group=pg))
            else:
                _wait(dist.irecv(buf, a, group=pg), self.p2p.timeout if staged else None,
                      f'relay link handshake with rank {a}')
        for w in works:
            _wait(w, self.p2p.timeout if staged else None, 'relay link handshake')
        if where.type == 'cuda':
            torch.cuda.synchronize(where)

    # -- backward ---------------------------------------------------------------------------

    def backward(self, losses: Optional[Sequence[Tensor]] = None) -> None:
        """Back-propagate every micro-batch (reverse order) and ship input gradients.

        The last stage passes one scalar loss per micro-batch; the others pass
        ``None``.
        """
        # split weight-gradient reductions of the fused ops are deferred to one flush after
        # the last micro-batch (ops/gradacc.py deferred_wgrad), issued once every stream
        # that wrote a slab has been joined to the current one
        from torchgpipe_amd.ops.gradacc import deferred_wgrad
        with deferred_wgrad(self.device, self.device.type == 'cuda'):
            self._backward(losses)
            if self.device.type == 'cuda':
                # a caller's ops.convbn.wgrad_stream_scope: its side stream wrote slabs
                from torchgpipe_amd.ops.convbn import join_wgrad_stream
                join_wgrad_stream(self.device)

    def _backward(self, losses: Optional[Sequence[Tensor]] = None) -> None:
        if self._recompute_lanes() is not None or self._fwd_lanes is not None:
            with _shared_accumulators():
                self._backward_cells(losses)
        else:
            self._backward_cells(losses)

    def _backward_cells(self, losses: Optional[Sequence[Tensor]] = None) -> None:
        if self.is_last and losses is None:
            raise ValueError('the last stage must pass the per-micro-batch losses')
        nxt = self.ranks[self.rank + 1] if not self.is_last else None
        prev = self.ranks[self.rank - 1] if self.rank > 0 else None
        me = self.ranks[self.rank]

        cells = list(reversed(self._cells))
        lanes = self._recompute_lanes()
        on_gpu = self.device.type == 'cuda'
        main = torch.cuda.current_stream(self.device) if on_gpu else None
        seg = self._segments if self._seg_phase in ('capture', 'replay') else None
        # recomputations on two lanes update running statistics concurrently: slotted, and
        # folded in the order they were issued (the reference's backward order)
        self._rec_slotted = lanes is not None and seg is None and self._stat_slots is not None
        if self._rec_slotted:
            assert self._stat_slots is not None
            self._stat_slots.begin(len(cells))
        # the capture step recomputes no cell ahead: a graph captured while another cell's
        # autograd graph is alive would share its AccumulateGrad nodes (and their streams)
        ahead = seg is None or self._seg_phase == 'replay'
        persistent = self._persistent
        # backward_thread: the previous micro-batch's backward, still being enqueued by the
        # helper thread (future, cell, stream); joined before the next one's starts
        threaded = self.backward_thread and self._probe is None
        try:
            pending = self._backward_loop(cells, losses, lanes, main, seg, ahead, persistent,
                                          threaded, nxt, prev, me)
        except BaseException:
            self._drain_pool()  # no backward left running into the next step
            raise
        if pending is not None:
            self._finish_pending(pending, me, prev)
        if on_gpu:
            # fused kernels on the lanes wrote .grad without autograd knowing
            cur = torch.cuda.current_stream(self.device)
            for lane in (lanes or []) + (self._fwd_lanes or []):
                cur.wait_stream(lane)
        if self._rec_slotted:
            assert self._stat_slots is not None
            self._stat_slots.commit()
            self._rec_slotted = False
        if seg is not None:
            seg.end_backward()
        if self._cache_state == 'measuring':
            size_cache_budget(self.device, torch.cuda.max_memory_allocated(self.device))
            self._cache_state = 'sized'
        self._cells = []
        self.p2p.flush()
        self._stripe_end()

    def _finish_pending(self, pending: Tuple[Any, _Cell, Optional[torch.cuda.Stream],
                                             Optional[Tuple[Tensor, ...]]],
                        me: int, prev: Optional[int]) -> None:
        """Join a helper-thread backward and ship its input gradients (on the recomputed
        leaves when it back-propagated through the recomputed graph)."""
        fut, cell, run, leaves = pending
        fut.result()
        if leaves is None:
            self._ship_input_grads(cell, run, None, me, prev)
        else:
            self._ship_input_grads(cell, run, [self._grad_of(x) for x in leaves], me, prev,
                                   on_run=False)

    def _drain_pool(self) -> None:
        if self._bwd_pool is not None:
            self._bwd_pool.shutdown(wait=True)
            self._bwd_pool = None

    def _backward_loop(self, cells: List[_Cell], losses: Optional[Sequence[Tensor]],
                       lanes: Optional[List[torch.cuda.Stream]],
                       main: Optional[torch.cuda.Stream], seg: Optional[Any], ahead: bool,
                       persistent: bool, threaded: bool, nxt: Optional[int],
                       prev: Optional[int], me: int
                       ) -> Optional[Tuple[Any, _Cell, Optional[torch.cuda.Stream],
                                           Optional[Tuple[Tensor, ...]]]]:
        """Steps 1-4 of every micro-batch's backward (``_backward_cells``); returns the
        last micro-batch's backward when the helper thread still owns it."""
        prev_run: Optional[torch.cuda.Stream] = None
        pending: Optional[Tuple[Any, _Cell, Optional[torch.cuda.Stream],
                                Optional[Tuple[Tensor, ...]]]] = None
        for j, cell in enumerate(cells):
            i = cell.index
            # 1. post the gradient receives first ...
            grad_msg = None
            if nxt is not None and any(t.requires_grad for t in cell.outputs[:cell.n_act_out]):
                grad_msg = self.p2p.recv(nxt, self._key('gact', i, nxt, me),
                                         persistent=persistent)
            skip_grad_msgs = []
            for dst in sorted({d for d, _ in self.out_skips}):
                peer = self.ranks[dst]
                skip_grad_msgs.append(
                    (dst, self.p2p.recv(peer, self._key('gskip', i, peer, me),
                                        persistent=persistent)))
            # 2. ... then recompute while they are in flight
            if lanes is None:
                if cell.seg:
                    assert seg is not None and main is not None
                    with trace.range(f'recompute graph mb{i} stage{self.rank}'):
                        seg.recompute(i, cell.fn, main)
                elif cell.chk is not None:
                    with trace.range(f'recompute mb{i} stage{self.rank}'):
                        cell.chk.recompute_now()
            else:
                assert main is not None
                self._recompute_on_lane(cell, lanes[j % 2], main)
                if j + 1 < len(cells) and ahead:
                    # the next micro-batch's recomputation (which touches no gradient) runs
                    # on the other lane while this backward runs; issued before this
                    # cell's gradient wait so it never queues behind the transfer
                    self._recompute_on_lane(cells[j + 1], lanes[(j + 1) % 2], main)

            if pending is not None:
                # the previous micro-batch's backward has been enqueued: ship its gradients
                self._finish_pending(pending, me, prev)
                pending = None

            # 3. backward through this cell -- a recomputed one straight through the
            #    recomputed graph (its Checkpoint node's reentrant backward would wrap the
            #    same work in a second engine call: 0.7 ms of host per AmoebaNet micro-batch)
            tensors: List[Tensor] = []
            grads: List[Tensor] = []
            direct = bool(self.direct_backward and cell.chk is not None and not cell.seg
                          and cell.chk.shared.recomputed)
            rec_out: Tuple[Tensor, ...] = ()
            leaves: Tuple[Tensor, ...] = ()
            if direct:
                assert cell.chk is not None
                rec_out, leaves = cell.chk.take_recomputed()
            # captured cells: the gradient of each output (None: none), and whether it sits
            # in a persistent receive buffer
            seg_grads: List[Optional[Tensor]] = [None] * len(cell.outputs)
            seg_kept = [False] * len(cell.outputs)
            act_out = cell.outputs[:cell.n_act_out]
            mark = self._probe_begin() if grad_msg is not None or skip_grad_msgs else None
            if self.is_last:
                assert losses is not None
                if cell.seg:  # the loss gradient w.r.t. the cell's output leaves
                    torch.autograd.backward([losses[i]], [torch.ones_like(losses[i])])
                    for k, t in enumerate(act_out):
                        seg_grads[k] = t.grad
                elif direct:
                    # the loss's gradient w.r.t. the cell's outputs (a backward through the
                    # loss alone), then on into the recomputed graph; leaves the loss reaches
                    # around the outputs (a learnable loss head) get theirs in the same pass
                    ks = [k for k, t in enumerate(act_out) if t.requires_grad]
                    outs = [act_out[k] for k in ks]
                    extra = _loss_leaves(losses[i], outs)
                    grads_all = torch.autograd.grad([losses[i]], outs + extra,
                                                    [torch.ones_like(losses[i])],
                                                    allow_unused=True)
                    gouts = grads_all[:len(outs)]
                    with torch.no_grad():
                        for leaf, g in zip(extra, grads_all[len(outs):]):
                            if g is None:
                                continue
                            if leaf.grad is None:
                                leaf.grad = g.detach().clone()
                            else:
                                leaf.grad += g
                    for k, g in zip(ks, gouts):
                        if g is not None and rec_out[k].requires_grad:
                            tensors.append(rec_out[k])
                            grads.append(g)
                else:
                    tensors.append(losses[i])
                    grads.append(torch.ones_like(losses[i]))
            elif grad_msg is not None:
                received = iter(grad_msg.wait())
                for k, t in enumerate(act_out):
                    if t.requires_grad:
                        g = next(received)
                        if direct:
                            if rec_out[k].requires_grad:
                                tensors.append(rec_out[k])
                                grads.append(g)
                            continue
                        tensors.append(t)
                        grads.append(g)
                        seg_grads[k], seg_kept[k] = grads[-1], persistent
            skip_out = cell.outputs[cell.n_act_out:]
            dst_of = [d for d, _ in self.out_skips]
            for dst, msg in skip_grad_msgs:
                received = iter(msg.wait())
                for k, (d, t) in enumerate(zip(dst_of, skip_out)):
                    if d == dst:
                        g = next(received)
                        if direct:
                            r = rec_out[cell.n_act_out + k]
                            if t.requires_grad and r.requires_grad:
                                tensors.append(r)
                                grads.append(g)
                            continue
                        if t.requires_grad:
                            tensors.append(t)
                            grads.append(g)
                            seg_grads[cell.n_act_out + k] = g
                            seg_kept[cell.n_act_out + k] = persistent
            self._probe_end('bwd', mark)
            # A cell computed or recomputed on a lane runs its backward there (autograd
            # replays each op on its forward stream).  Order it after main (received
            # gradients, the loss) and after the previous micro-batch's backward,
            # whichever stream ran it: the fused ops add into the same .grad buffers
            # outside autograd, so nothing else would order the two.
            run = cell.lane if cell.lane is not None else main
            if cell.lane is not None:
                assert main is not None
                cell.lane.wait_stream(main)
            if run is not None and prev_run is not None and prev_run is not run:
                run.wait_stream(prev_run)
            gins: Optional[List[Tensor]] = None
            if cell.seg:
                assert seg is not None and run is not None
                with trace.range(f'bwd graph mb{i} stage{self.rank}'):
                    gins = seg.backward(i, seg_grads, seg_kept, run)
            elif threaded and tensors:
                # enqueued by the helper thread while this thread goes on to the next
                # micro-batch's receives and recomputation (joined there, before its
                # backward: the fused ops add into the same .grad buffers)
                pending = (self._backward_pool().submit(
                    self._threaded_backward, tensors, grads, main, i), cell, run,
                    leaves if direct else None)
                prev_run = run
                continue
            else:
                with trace.range(f'bwd mb{i} stage{self.rank}'):
                    if tensors:
                        torch.autograd.backward(tensors, grads)
            prev_run = run
            if direct:
                # the input gradients sit on the recomputation's leaves
                gins = [self._grad_of(x) for x in leaves]
                del rec_out, leaves, tensors, grads

            # 4. ship input gradients upstream
            self._ship_input_grads(cell, run, gins, me, prev, on_run=not direct)
        return pending

    def _ship_input_grads(self, cell: _Cell, run: Optional[torch.cuda.Stream],
                          gins: Optional[List[Tensor]], me: int, prev: Optional[int],
                          on_run: bool = True) -> None:
        """Send a micro-batch's input gradients upstream (a replayed backward ran no
        autograd, so its sends leave from the stream that ran it; gradients ``gins`` that
        autograd accumulated leave from the current stream, which the engine synced) and
        release the cell."""
        i = cell.index
        n_in_act = len(cell.inputs) - len(self.in_skips)

        def grad_in(k: int) -> Tensor:
            return gins[k] if gins is not None else self._grad_of(cell.inputs[k])

        with torch.cuda.stream(run) if gins is not None and on_run and run is not None \
                else contextlib.nullcontext():
            if prev is not None:
                gin = [grad_in(k) for k in range(n_in_act) if cell.inputs[k].requires_grad]
                self.p2p.send(gin, prev, self._key('gact', i, me, prev))
            by_src: Dict[int, List[Tensor]] = {}
            for k, (src, _) in enumerate(self.in_skips):
                by_src.setdefault(src, []).append(grad_in(n_in_act + k))
            for src in sorted(by_src):
                peer = self.ranks[src]
                self.p2p.send(by_src[src], peer, self._key('gskip', i, me, peer))
        cell.inputs = []
        cell.outputs = []
        cell.chk = None
        cell.lane = None
        cell.fn = None

    def _backward_pool(self) -> Any:
        if self._bwd_pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._bwd_pool = ThreadPoolExecutor(1, thread_name_prefix='tgpipe-bwd')
        return self._bwd_pool

    def _threaded_backward(self, tensors: List[Tensor], grads: List[Tensor],
                           stream: Optional[torch.cuda.Stream], i: int) -> None:
        """``torch.autograd.backward`` on the helper thread, with the caller's device and
        current stream (the engine syncs the incoming gradients with it)."""
        with contextlib.ExitStack() as ctx:
            if stream is not None:
                ctx.enter_context(torch.cuda.device(self.device))
                ctx.enter_context(torch.cuda.stream(stream))
            with trace.range(f'bwd mb{i} stage{self.rank}'):
                torch.autograd.backward(tensors, grads)

    def _recompute_lanes(self) -> Optional[List[torch.cuda.Stream]]:
        if not self.overlap_recompute or self.device.type != 'cuda':
            return None
        if torch.cuda.is_current_stream_capturing():
            # the recompute lanes stay out of hipGraph captures (parallel/graph.py): only the
            # two-stream cells are verified inside captures (profiles/r3/capture_crash.md)
            return None
        if self._lanes is None:
            self._lanes = [named_stream(self.device, 'recompute-lane0'),
                           named_stream(self.device, 'recompute-lane1')]
        return self._lanes

    def _forward_lanes(self) -> Optional[List[torch.cuda.Stream]]:
        """Two streams for the forward micro-batches of a stateless partition.

        Micro-batch i runs on lane i % 2 after main (which holds its received inputs), and
        its outputs are sent from that lane, so consecutive micro-batches overlap whenever
        their inputs are already here: on the first stage, and on a stage slower than its
        upstream (the pipeline's bottleneck, where inputs queue).  Partitions with running
        statistics (BatchNorm) take them when ``_lanes_ok``: their updates are slotted and
        folded in micro-batch order (:class:`~torchgpipe_amd.runstats.OrderedRunningStats`).
        """
        if not self.overlap_forward or not self._lanes_ok():
            return None
        if self.device.type != 'cuda' or torch.cuda.is_current_stream_capturing():
            return None
        if self._fwd_lanes is None:
            self._fwd_lanes = [named_stream(self.device, 'forward-lane0'),
                               named_stream(self.device, 'forward-lane1')]
        return self._fwd_lanes

    def _lanes_ok(self) -> bool:
        """Whether this partition's forwards may overlap: stateless, or running statistics
        that can be slotted and no multi-stream cells (AmoebaNet's side streams are shared
        process-wide, so two lanes' cells would interleave on them)."""
        if not self._stateful:
            return True
        if self._stat_slots is None:
            return False
        return not any(isinstance(getattr(m, 'streams', 0), int) and getattr(m, 'streams', 0)
                       for m in self.partition.modules())

    def _recompute_on_lane(self, cell: _Cell, lane: torch.cuda.Stream,
                           main: torch.cuda.Stream) -> None:
        """Issue ``cell``'s recomputation on ``lane`` (once); its backward then runs there."""
        if cell.seg:
            if cell.lane is None:
                assert self._segments is not None
                with trace.range(f'recompute graph mb{cell.index} stage{self.rank}'):
                    self._segments.recompute(cell.index, cell.fn, lane)
                cell.lane = lane
            return
        if cell.chk is None or cell.lane is not None:
            return
        lane.wait_stream(main)
        for t in cell.inputs:
            t.record_stream(lane)
        slots = self._stat_slots if self._rec_slotted else None
        with torch.cuda.stream(lane), trace.range(f'recompute mb{cell.index} stage{self.rank}'), \
                slots.update() if slots is not None else contextlib.nullcontext():
            cell.chk.recompute_now()
        cell.lane = lane

    # -- diagnostics ------------------------------------------------------------------------

    def _streams(self) -> List[torch.cuda.Stream]:
        return ([torch.cuda.current_stream(self.device)] + list(self._lanes or [])
                + list(self._fwd_lanes or []))

    def _probe_begin(self) -> Any:
        """Marker before a receive wait: events on main and every lane (GPU), or the host
        clock (host-blocking transports)."""
        if self._probe is None:
            return None
        if self.device.type == 'cuda':
            events = []
            for s in self._streams():
                e = torch.cuda.Event(enable_timing=True)
                e.record(s)
                events.append(e)
            return events
        return time.perf_counter()

    def _probe_end(self, kind: str, mark: Any) -> None:
        if self._probe is None or mark is None:
            return
        if self.device.type == 'cuda':
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.device))
            self._probe.append((kind, mark, e))
        else:
            self._probe.append((kind, mark, time.perf_counter()))

    def probe_step(self, step: Callable[[], Any]) -> Dict[str, float]:
        """Run ``step()`` (one training step of this stage) with its receive waits timed.

        Returns, in ms: ``step_ms`` (the step on this rank, from the first kernel it queues
        to the last), ``fwd_wait_ms`` / ``bwd_wait_ms`` (time every stream of this stage
        sat idle waiting for activations / gradients to arrive: each wait is measured from
        the moment the last of main and the lanes reached it, so lane compute is not
        counted), ``fill_ms`` / ``drain_ms`` (the first forward and first backward wait:
        the pipeline fill and drain bubbles this rank sees), ``busy_ms`` (``step_ms``
        minus the waits) and ``host_enqueue_ms`` (host time until ``step()`` returned:
        Python, autograd and launches -- above ``busy_ms`` the rank is launch-bound).
        Meant for one diagnostic step outside the timed ones: the events add a little host
        work per micro-batch.
        """
        gpu = self.device.type == 'cuda'
        self._probe = []
        try:
            if gpu:
                torch.cuda.synchronize(self.device)
                start = torch.cuda.Event(enable_timing=True)
                start.record(torch.cuda.current_stream(self.device))
                h0 = time.perf_counter()
                step()
                host = 1000 * (time.perf_counter() - h0)
                end = torch.cuda.Event(enable_timing=True)
                end.record(torch.cuda.current_stream(self.device))
                for s in self._streams():
                    torch.cuda.current_stream(self.device).wait_stream(s)
                torch.cuda.synchronize(self.device)
                total = start.elapsed_time(end)

                def wait_of(mark: Any, stop: Any) -> float:
                    began = max(start.elapsed_time(e) for e in mark)
                    return max(0.0, start.elapsed_time(stop) - began)
            else:
                t0 = time.perf_counter()
                step()
                total = host = 1000 * (time.perf_counter() - t0)

                def wait_of(mark: Any, stop: Any) -> float:
                    return 1000 * (stop - mark)
            waits = [(kind, wait_of(m, e)) for kind, m, e in self._probe]
        finally:
            self._probe = None
        fwd = [w for k, w in waits if k == 'fwd']
        bwd = [w for k, w in waits if k == 'bwd']
        return {'step_ms': round(total, 3),
                'fwd_wait_ms': round(sum(fwd), 3), 'bwd_wait_ms': round(sum(bwd), 3),
                'fill_ms': round(fwd[0], 3) if fwd else 0.0,
                'drain_ms': round(bwd[0], 3) if bwd else 0.0,
                'busy_ms': round(total - sum(fwd) - sum(bwd), 3),
                'host_enqueue_ms': round(host, 3)}

    @staticmethod
    def _grad_of(t: Tensor) -> Tensor:
        return t.grad if t.grad is not None else torch.zeros_like(t)

    # -- convenience ------------------------------------------------------------------------

    def train_step(self, input: Optional[TensorOrTensors], target: Optional[Tensor],
                   loss_fn: Callable[[Tensor, Tensor], Tensor], *,
                   signature: Optional[Signature] = None) -> Optional[Tensor]:
        """Forward + backward of one mini-batch; returns the mean loss on the last stage.

        ``loss_fn(output, target)`` must be a mean-reduced loss; per-micro-batch
        losses are weighted by micro-batch size so the gradient equals the
        full-batch gradient of the reference (loss on the gathered output).
        """
        outputs = self.forward(input, signature=signature)
        if not self.is_last:
            self.backward(None)
            return None
        assert target is not None
        targets = target.chunk(self.chunks)
        total = float(target.size(0))
        losses = [loss_fn(out, tgt) * (tgt.size(0) / total)  # type: ignore[arg-type]
                  for out, tgt in zip(outputs, targets)]
        self.backward(losses)
        with torch.no_grad():
            return torch.stack([l.detach() for l in losses]).sum()
