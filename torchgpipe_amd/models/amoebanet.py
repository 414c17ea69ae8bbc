"""AmoebaNet-D as a flat ``nn.Sequential`` (benchmark model).

Same architecture as the reference benchmark model
(``benchmarks/models/amoebanet/__init__.py:138-194``, ``operations.py``,
``genotype.py``): a ReLU-Conv-BN stem, two reduction cells, then three
stacks of ``L/3`` normal cells separated by reduction cells, and a classifier.
Cells exchange ``(x, skip)`` tuples, so pipeline boundaries carry two tensors.
AmoebaNet-D(18, 256) = 24 layers, 122.47 M parameters; the reference balance
tables (``benchmarks/amoebanetd-speed/main.py:35-96``) apply unchanged.

Kept quirks of the reference for benchmark fidelity: the normal-cell concat is
TensorFlow's ``[0, 3, 4, 6]``, and ``max_pool_3x3`` is an average pool
(``operations.py:57-59`` in the reference).

MI355X path: every ReLU → Conv(1×1 / 1×7 / 7×1) → BatchNorm triplet is an
``ops.convbn`` fused op (implicit-GEMM fp32 MFMA kernel with the ReLU on its
operand load and the BatchNorm statistics in its epilogue), FactorizedReduce is
one fused op over both shifted branches, and the ``left + right`` sum of each
cell node is folded into the right branch's normalisation pass.  The modules
keep the reference's children, so parameters and state-dict keys are the same
as the plain model (``fused=False``), which also serves as the numerics oracle.
"""
from collections import OrderedDict
import contextlib
import os
import threading
from typing import Callable, Dict, Iterator, List, Optional, Tuple, Union

import torch
from torch import Tensor, nn

from torchgpipe_amd.ops.convbn import (FusedChain, ReLUConvBN, _GroupCache, fusable,
                                       fused_triplets, group_relu_conv_bn, groupable,
                                       relu_conv_bn)
from torchgpipe_amd.ops.pool import AvgPool3x3
from torchgpipe_amd.ops.unet_ops import MaxPool2x2

__all__ = ['amoebanetd', 'NORMAL_OPERATIONS', 'REDUCTION_OPERATIONS', 'set_cell_streams']

_SIDE_STREAMS: Dict[Tuple[torch.device, int, int], torch.cuda.Stream] = {}
_CAPTURE_STREAMS = os.environ.get('TGPIPE_CAPTURE_STREAMS', '1') != '0'
# TGPIPE_SHARE_POOLS=0 computes a cell's duplicate average pools twice (Cell._shared_plan)
_SHARE_POOLS = os.environ.get('TGPIPE_SHARE_POOLS', '1') != '0'
# streams per cell for set_cell_streams(model, True) (TGPIPE_CELL_STREAMS)
DEFAULT_CELL_STREAMS = int(os.environ.get('TGPIPE_CELL_STREAMS', '3'))
# at most this many inside a whole-step hipGraph capture (StepGraph): a capture holding a
# three-stream forward and its backward segfaults inside the runtime, even for one
# micro-batch; per-pass captures (PipelineStage(graph_cells=True)) keep the eager stream
# count (profiles/r3/capture_crash.md, round-4 section)
CAPTURE_CELL_STREAMS = int(os.environ.get('TGPIPE_CAPTURE_CELL_STREAMS', '2'))
_WHOLE_STEP = threading.local()


@contextlib.contextmanager
def whole_step_capture() -> Iterator[None]:
    """Mark a capture that records forward and backward in one graph (StepGraph): cells
    then use at most ``CAPTURE_CELL_STREAMS`` streams."""
    prev = getattr(_WHOLE_STEP, 'on', False)
    _WHOLE_STEP.on = True
    try:
        yield
    finally:
        _WHOLE_STEP.on = prev


def _side_stream(device: torch.device, main: torch.cuda.Stream, index: int = 1
                 ) -> torch.cuda.Stream:
    """Side stream ``index`` paired with ``main``: a cell recomputed on a pipeline's
    recompute lane (``PipelineStage(overlap_recompute=True)``) gets its own, so its branch
    work does not queue behind the backward of the micro-batch running beside it."""
    key = (device, main.stream_id, index)
    stream = _SIDE_STREAMS.get(key)
    if stream is None:
        stream = _SIDE_STREAMS[key] = torch.cuda.Stream(device)
    return stream


def prepare_side_streams(device: torch.device, main: torch.cuda.Stream,
                         count: int = 4) -> None:
    """Create the side streams paired with ``main`` ahead of time (``StepGraph`` calls it for
    its capture stream, so no stream is created inside a capture)."""
    for i in range(1, count):
        _side_stream(torch.device(device), main, i)


class _JoinSideInBackward(torch.autograd.Function):
    """Identity on the cell inputs whose backward makes the current stream wait for the side
    streams: the fused ops on a side stream write ``param.grad`` themselves (gradient-
    accumulation fusion), which autograd's end-of-backward stream sync does not see.  Every
    op of the cell lies upstream of the inputs' gradients, so this backward runs after all
    of them have been issued."""

    @staticmethod
    def forward(ctx, streams: List[torch.cuda.Stream], *xs: Tensor):  # type: ignore[override]
        ctx.streams = streams
        return tuple(x.view_as(x) for x in xs)

    @staticmethod
    def backward(ctx, *grads: Tensor):  # type: ignore[override]
        current = torch.cuda.current_stream()
        for stream in ctx.streams:
            current.wait_stream(stream)
        return (None,) + grads


def _op_cost_module(m: nn.Module) -> float:
    if isinstance(m, FusedChain):
        return float(sum(isinstance(c, nn.Conv2d) for c in m.children()))
    if isinstance(m, FactorizedReduce):
        return 1.0
    return 0.0


def _op_cost(op: 'Operation') -> float:
    """Rough relative device time of a cell operation (number of convolutions)."""
    m = op.module
    if isinstance(m, FusedChain):
        return float(sum(isinstance(c, nn.Conv2d) for c in m.children()))
    if isinstance(m, FactorizedReduce):
        return 1.0
    if isinstance(m, nn.Identity):
        return 0.0
    return 0.5  # pools


class Operation(nn.Module):
    def __init__(self, name: str, module: nn.Module) -> None:
        super().__init__()
        self.name = name
        self.module = module

    def __repr__(self) -> str:
        return f'Operation[{self.name}]'

    @property
    def takes_add(self) -> bool:
        """Whether ``add`` folds into the module's own last pass (no separate add)."""
        return isinstance(self.module, (FusedChain, FactorizedReduce, AvgPool3x3, MaxPool2x2))

    def forward(self, x: Tensor, add: Optional[Tensor] = None,  # type: ignore[override]
                first: Optional[Tensor] = None) -> Tensor:
        """``module(x)``, plus ``add`` (folded into a fused op's last pass when it can).
        ``first``: the output of the module's first (ReLU, Conv, BN) triplet, computed by a
        grouped op (``Cell``) -- the chain continues from there."""
        if first is not None:
            assert isinstance(self.module, FusedChain)
            if len(self.module) == 3:  # a single triplet: that is the result
                return first if add is None else first + add
            return self.module(first, add, start=1)
        if add is not None and self.takes_add:
            return self.module(x, add)
        out = self.module(x)
        return out if add is None else out + add


def conv_bn_chain(*modules: nn.Module) -> nn.Sequential:
    return FusedChain(*modules)


def _relu_conv_bn(cin: int, cout: int, kernel=1, stride=1, padding=0) -> nn.Sequential:  # type: ignore[no-untyped-def]
    return ReLUConvBN(nn.ReLU(inplace=False),
                      nn.Conv2d(cin, cout, kernel, stride, padding, bias=False),
                      nn.BatchNorm2d(cout))


class FactorizedReduce(nn.Module):
    """Stride-2 reduction via two offset 1×1 convs concatenated on channels."""

    def __init__(self, cin: int, cout: int) -> None:
        super().__init__()
        self.relu = nn.ReLU(inplace=False)
        self.pad = nn.ZeroPad2d((0, 1, 0, 1))
        self.conv1 = nn.Conv2d(cin, cout // 2, kernel_size=1, stride=2, bias=False)
        self.conv2 = nn.Conv2d(cin, cout // 2, kernel_size=1, stride=2, bias=False)
        self.bn = nn.BatchNorm2d(cout)

    def forward(self, x: Tensor, add: Optional[Tensor] = None) -> Tensor:  # type: ignore[override]
        if fusable(x, [self.conv1, self.conv2], self.bn):
            # both strided branches in one op: the second reads x shifted by one pixel
            # (the zero pad of the reference falls out of the bounds check)
            return relu_conv_bn(x, [(self.conv1, 0), (self.conv2, 1)], self.bn, add=add)
        x = self.relu(x)
        shifted = self.pad(x[:, :, 1:, 1:])
        out = self.bn(torch.cat([self.conv1(x), self.conv2(shifted)], dim=1))
        return out if add is None else out + add


def op_none(c: int, stride: int) -> Operation:
    return Operation('none', nn.Identity() if stride == 1 else FactorizedReduce(c, c))


def op_avg_pool_3x3(c: int, stride: int) -> Operation:
    return Operation('avg_pool_3x3', AvgPool3x3(stride))


def op_max_pool_3x3(c: int, stride: int) -> Operation:
    # Reference quirk: implemented as an average pool.
    return Operation('max_pool_3x3', AvgPool3x3(stride))


def op_max_pool_2x2(c: int, stride: int) -> Operation:
    # stride 2 (every use in the genotypes) on the index-free HIP kernel (ops/unet_ops.py)
    pool = MaxPool2x2() if stride == 2 else nn.MaxPool2d(2, stride=stride, padding=0)
    return Operation('max_pool_2x2', pool)


def _bottleneck(c: int, middle: List[nn.Module]) -> nn.Sequential:
    q = c // 4
    return conv_bn_chain(nn.ReLU(inplace=False), nn.Conv2d(c, q, 1, bias=False),
                         nn.BatchNorm2d(q), *middle,
                         nn.ReLU(inplace=False), nn.Conv2d(q, c, 1, bias=False),
                         nn.BatchNorm2d(c))


def op_conv_1x7_7x1(c: int, stride: int) -> Operation:
    q = c // 4
    middle: List[nn.Module] = [
        nn.ReLU(inplace=False),
        nn.Conv2d(q, q, (1, 7), stride=(1, stride), padding=(0, 3), bias=False),
        nn.BatchNorm2d(q),
        nn.ReLU(inplace=False),
        nn.Conv2d(q, q, (7, 1), stride=(stride, 1), padding=(3, 0), bias=False),
        nn.BatchNorm2d(q),
    ]
    return Operation('conv_1x7_7x1', _bottleneck(c, middle))


def op_conv_1x1(c: int, stride: int) -> Operation:
    return Operation('conv_1x1', _relu_conv_bn(c, c, 1, stride))


def op_conv_3x3(c: int, stride: int) -> Operation:
    q = c // 4
    middle: List[nn.Module] = [nn.ReLU(inplace=False),
                               nn.Conv2d(q, q, 3, stride=stride, padding=1, bias=False),
                               nn.BatchNorm2d(q)]
    return Operation('conv_3x3', _bottleneck(c, middle))


OpFactory = Callable[[int, int], Operation]

# AmoebaNet-D genotype: (input state index, operation) pairs, two per node.
NORMAL_OPERATIONS: List[Tuple[int, OpFactory]] = [
    (1, op_conv_1x1), (1, op_max_pool_3x3),
    (1, op_none), (0, op_conv_1x7_7x1),
    (0, op_conv_1x1), (0, op_conv_1x7_7x1),
    (2, op_max_pool_3x3), (2, op_none),
    (1, op_avg_pool_3x3), (5, op_conv_1x1),
]
NORMAL_CONCAT = [0, 3, 4, 6]

REDUCTION_OPERATIONS: List[Tuple[int, OpFactory]] = [
    (0, op_max_pool_2x2), (0, op_max_pool_3x3),
    (2, op_none), (1, op_conv_3x3),
    (2, op_conv_1x7_7x1), (2, op_max_pool_3x3),
    (3, op_none), (1, op_max_pool_2x2),
    (2, op_avg_pool_3x3), (3, op_conv_1x1),
]
REDUCTION_CONCAT = [4, 5, 6]


class Classify(nn.Module):
    def __init__(self, channels_prev: int, num_classes: int) -> None:
        super().__init__()
        self.pool = nn.AvgPool2d(7)
        self.flat = nn.Flatten()
        self.fc = nn.Linear(channels_prev, num_classes)

    def forward(self, states: Tuple[Tensor, Tensor]) -> Tensor:  # type: ignore[override]
        x, _ = states
        return self.fc(self.flat(self.pool(x)))


class Stem(nn.Module):
    def __init__(self, channels: int) -> None:
        super().__init__()
        self.relu = nn.ReLU(inplace=False)
        self.conv = nn.Conv2d(3, channels, 3, stride=2, padding=1, bias=False)
        self.bn = nn.BatchNorm2d(channels)

    def forward(self, x: Tensor) -> Tensor:  # type: ignore[override]
        if fusable(x, [self.conv], self.bn):
            return relu_conv_bn(x, [(self.conv, 0)], self.bn)
        return self.bn(self.conv(self.relu(x)))


class Cell(nn.Module):
    def __init__(self, c_prev_prev: int, c_prev: int, c: int, reduction: bool,
                 reduction_prev: bool) -> None:
        super().__init__()
        self.reduce1 = _relu_conv_bn(c_prev, c)
        self.reduce2: nn.Module = nn.Identity()
        if reduction_prev:
            self.reduce2 = FactorizedReduce(c_prev_prev, c)
        elif c_prev_prev != c:
            self.reduce2 = _relu_conv_bn(c_prev_prev, c)

        genotype = REDUCTION_OPERATIONS if reduction else NORMAL_OPERATIONS
        self.concat = REDUCTION_CONCAT if reduction else NORMAL_CONCAT
        self.indices = [i for i, _ in genotype]
        self.operations = nn.ModuleList(
            factory(c, 2 if reduction and i < 2 else 1) for i, factory in genotype)
        self.streams = 0
        self._group = self._group_plan()
        self._group_cache = _GroupCache()
        self._shared = self._shared_plan()
        self._plans: Dict[int, List[int]] = {}
        self._event_flags: Dict[int, List[bool]] = {}

    @property
    def _plan(self) -> List[int]:
        """The stream plan for the current stream count (two streams when off)."""
        return self._stream_plan(max(2, int(self.streams)))

    def _stream_plan(self, count: int = 2) -> List[int]:
        """Stream (0 = current, 1.. = side streams) of every node.

        List scheduling over ``count`` streams with a rough cost per node (convolutions):
        the two input reductions go to streams 0 and 1; every later node goes to the
        stream where it can start earliest after its inputs (ties: a stream one of its
        inputs ran on, then the lower index).  A grouped first-triplet op counts at the
        start of the node that runs it, and the nodes that consume its other outputs are
        ready once it is done -- with three streams the two 1x7-7x1 chains after it run
        side by side.
        """
        plan = self._plans.get(count)
        if plan is not None:
            return plan
        ops = list(self.operations)
        g_ops = self._group[1]
        plan = [0, min(1, count - 1)]
        finish = [_op_cost_module(self.reduce1), _op_cost_module(self.reduce2)]
        free = [0.0] * count
        free[plan[0]] = finish[0]
        free[plan[1]] = max(free[plan[1]], finish[1])
        group_done = shared_done = -1.0
        for k in range(0, len(ops), 2):
            pair = (k, k + 1)
            ins = [self.indices[k], self.indices[k + 1]]
            ready = max(finish[i] for i in ins)
            uses_group = any(o in g_ops for o in pair)
            uses_shared = any(o in self._shared for o in pair)
            if uses_group and group_done >= 0:
                ready = max(ready, group_done)
            if uses_shared and shared_done >= 0:
                ready = max(ready, shared_done)
            own = {plan[i] for i in ins}
            s = min(range(count), key=lambda c: (max(ready, free[c]), c not in own, c))
            t = max(ready, free[s])
            if uses_group and group_done < 0:
                t += 0.6 * len(g_ops)  # the grouped GEMM, run by this node
                group_done = t
            if uses_shared and shared_done < 0:
                t += 0.5  # the shared pool, run by this node
                shared_done = t
            for o in pair:
                if o in g_ops:
                    t += _op_cost(ops[o]) - 1.0
                elif o not in self._shared:
                    t += _op_cost(ops[o])
            plan.append(s)
            finish.append(t)
            free[s] = t
        self._plans[count] = plan
        return plan

    def _group_plan(self) -> Tuple[int, List[int]]:
        """(input node, operations) whose first (ReLU, 1x1 Conv, BN) triplets read the same
        node and can run as one grouped GEMM (a normal cell's node 0 feeds three: the two
        1x7-7x1 bottlenecks and the 1x1); (-1, []) if no node feeds two or more."""
        by_input: Dict[int, List[int]] = {}
        for k, op in enumerate(self.operations):
            m = op.module
            if not isinstance(m, FusedChain):
                continue
            trip = fused_triplets(m)
            if not trip:
                continue
            relu, conv, _ = trip[0]
            if relu and tuple(conv.kernel_size) == (1, 1) and tuple(conv.stride) == (1, 1) and \
                    tuple(conv.padding) == (0, 0) and conv.bias is None:
                by_input.setdefault(self.indices[k], []).append(k)
        best = max(by_input.items(), key=lambda kv: len(kv[1]), default=(-1, []))
        if len(best[1]) < 2:
            return -1, []
        return best[0], best[1][:3]

    def _shared_plan(self) -> List[int]:
        """Operations that compute the same function of the same node (the genotypes apply a
        3x3 stride-1 average pool to one node twice: the reference's ``max_pool_3x3`` is an
        average pool, ``operations.py:57-59``); the first of them is run once and its output
        reused, its partners folding it in as their node sum."""
        if not _SHARE_POOLS:
            return []
        seen: Dict[Tuple[int, int], List[int]] = {}
        for k, op in enumerate(self.operations):
            m = op.module
            if type(m) is AvgPool3x3:
                stride = m.stride if isinstance(m.stride, int) else m.stride[0]
                seen.setdefault((self.indices[k], stride), []).append(k)
        for ks in seen.values():
            # each must pair with an operation that folds a sum (its node's other half)
            if len(ks) >= 2 and all(self.operations[k ^ 1].takes_add and k ^ 1 not in ks
                                    for k in ks):
                return ks
        return []

    def _grouped(self, nodes: List[Tensor]) -> Dict[int, Tensor]:
        """First-triplet outputs of the grouped operations (empty when not applicable)."""
        node, ops = self._group
        if node < 0 or node >= len(nodes):
            return {}
        x = nodes[node]
        triplets = [self.operations[k].module._triplets()[0] for k in ops]  # type: ignore[index]
        if not groupable(x, triplets):
            return {}
        outs = group_relu_conv_bn(x, triplets, self._group_cache)
        return dict(zip(ops, outs))

    def extra_repr(self) -> str:
        return f'indices: {self.indices}'

    def _node(self, k: int, nodes: List[Tensor], pre: Optional[Dict[int, Tensor]] = None,
              shared: Optional[Dict[int, Tensor]] = None) -> Tensor:
        # node = left + right: run the operation that cannot fold a sum first and hand
        # its output to the other one's last pass (a shared operation's output, computed
        # once per cell, is always the one handed over)
        ops = self.operations
        pre = pre or {}
        if k in self._shared or k + 1 in self._shared:
            a = k if k in self._shared else k + 1
            b = a ^ 1
            assert shared is not None
            if a not in shared:
                out = ops[a](nodes[self.indices[a]])
                for j in self._shared:
                    shared[j] = out
            return ops[b](nodes[self.indices[b]], add=shared[a], first=pre.get(b))
        a, b = (k, k + 1) if ops[k + 1].takes_add or not ops[k].takes_add else (k + 1, k)
        first = ops[a](nodes[self.indices[a]], first=pre.get(a))
        return ops[b](nodes[self.indices[b]], add=first, first=pre.get(b))

    def forward(self, states: Union[Tensor, Tuple[Tensor, Tensor]]  # type: ignore[override]
                ) -> Tuple[Tensor, Tensor]:
        s1, s2 = states if isinstance(states, tuple) else (states, states)
        skip = s1
        # (also inside hipGraph captures: the replay crash of round 2 was the runtime's
        # recursive DAG walk overflowing the main thread's stack, now launched from a
        # big-stack thread, utils/bigstack.py; TGPIPE_CAPTURE_STREAMS=0 keeps captures on
        # one stream)
        if self.streams and s1.is_cuda and (_CAPTURE_STREAMS or
                                            not torch.cuda.is_current_stream_capturing()):
            return self._forward_streams(s1, s2), skip
        nodes = [self.reduce1(s1), self.reduce2(s2)]
        pre = self._grouped(nodes)
        shared: Dict[int, Tensor] = {}
        for k in range(0, len(self.operations), 2):
            nodes.append(self._node(k, nodes, pre, shared))
        return torch.cat([nodes[i] for i in self.concat], dim=1), skip

    def _forward_streams(self, s1: Tensor, s2: Tensor) -> Tensor:
        """The cell's independent nodes on ``self.streams`` HIP streams
        (``set_cell_streams``).

        Node k runs on stream ``plan[k]`` after waiting on the events of inputs produced on
        another stream (the grouped first-triplet op and a shared pool have events of
        their own, recorded right after them, so their consumers do not wait for the rest
        of the node that ran them); tensors crossing streams are ``record_stream``-ed so the
        caching allocator does not hand their memory out early.  Autograd runs each
        backward op on its forward op's stream.
        """
        count = max(2, int(self.streams))
        if getattr(_WHOLE_STEP, 'on', False) and torch.cuda.is_current_stream_capturing():
            count = max(2, min(count, CAPTURE_CELL_STREAMS))
        plan = self._stream_plan(count)
        current = torch.cuda.current_stream(s1.device)
        streams = [current] + [_side_stream(s1.device, current, i) for i in range(1, count)]
        used = sorted(set(plan))
        sides = [streams[i] for i in used if i != 0]
        if torch.is_grad_enabled() and (s1.requires_grad or s2.requires_grad):
            if s1 is s2:
                s1 = s2 = _JoinSideInBackward.apply(sides, s1)[0]
            else:
                s1, s2 = _JoinSideInBackward.apply(sides, s1, s2)
        for side in sides:
            side.wait_stream(current)
        events: List[Optional[torch.cuda.Event]] = []
        nodes: List[Tensor] = []
        pre: Dict[int, Tensor] = {}
        shared: Dict[int, Tensor] = {}
        special: Dict[str, Tuple[int, torch.cuda.Event]] = {}  # 'group' / 'shared' -> (stream, ev)
        # which nodes need an event (an input of a node on another stream, or a concat input
        # off the current stream): fixed per plan
        flags = self._event_flags.get(count)
        if flags is None:
            flags = [any(plan[j] != plan[k] for j in range(k + 1, len(plan))) or
                     (plan[k] != 0 and k in self.concat) for k in range(len(plan))]
            self._event_flags[count] = flags

        def event(key: object) -> torch.cuda.Event:
            # a fresh event: recording a new one costs 2.3 us of host, re-recording a
            # pending one 5.6 (benchmarks/host_cell.py)
            return torch.cuda.Event()

        def run(k: int, fn: Callable[[], Tensor], inputs: List[int],
                external: List[Tensor], waits: List[str]) -> None:
            s = plan[k]
            stream = streams[s]
            for i in inputs:
                if plan[i] != s:
                    ev = events[i]
                    assert ev is not None
                    stream.wait_event(ev)
                    nodes[i].record_stream(stream)
            for name in waits:
                src, ev = special[name]
                if src != s:
                    stream.wait_event(ev)
                    for t in (pre.values() if name == 'group' else shared.values()):
                        t.record_stream(stream)
            if s != 0:
                for t in external:
                    t.record_stream(stream)
                # set / restore the current stream directly: a torch.cuda.stream block
                # costs 6.1 us of host, the two switches 0.9 (benchmarks/host_cell.py)
                torch.cuda.set_stream(stream)
                try:
                    out = fn()
                finally:
                    torch.cuda.set_stream(current)
            else:
                out = fn()
            ev = None
            if flags[k]:
                ev = event(k)
                ev.record(stream)
            nodes.append(out)
            events.append(ev)

        run(0, lambda: self.reduce1(s1), [], [s1], [])
        run(1, lambda: self.reduce2(s2), [], [s2], [])
        g_ops = self._group[1]
        for k in range(0, len(self.operations), 2):
            node = len(nodes)
            pair = (k, k + 1)
            ins = [self.indices[k], self.indices[k + 1]]
            waits: List[str] = []
            first_group = any(o in g_ops for o in pair) and 'group' not in special
            first_shared = any(o in self._shared for o in pair) and 'shared' not in special
            if any(o in g_ops for o in pair) and not first_group:
                waits.append('group')
            if any(o in self._shared for o in pair) and not first_shared:
                waits.append('shared')

            def fn(k: int = k, node: int = node, first_group: bool = first_group,
                   first_shared: bool = first_shared) -> Tensor:
                stream = streams[plan[node]]
                if first_group:
                    pre.update(self._grouped(nodes))
                    ev = event('group')
                    ev.record(stream)
                    special['group'] = (plan[node], ev)
                if first_shared:
                    a = next(o for o in (k, k + 1) if o in self._shared)
                    out = self.operations[a](nodes[self.indices[a]])
                    for j in self._shared:
                        shared[j] = out
                    ev = event('shared')
                    ev.record(stream)
                    special['shared'] = (plan[node], ev)
                return self._node(k, nodes, pre, shared)
            run(node, fn, ins, [], waits)
        for side in sides:
            streams[0].wait_stream(side)
        for i in self.concat:
            if plan[i] != 0:
                nodes[i].record_stream(streams[0])
        return torch.cat([nodes[i] for i in self.concat], dim=1)


def set_cell_streams(model: nn.Module, enabled: Union[bool, int] = True) -> None:
    """Run every AmoebaNet cell's independent nodes on several HIP streams (GPU inputs):
    ``True`` = ``DEFAULT_CELL_STREAMS`` (3, ``TGPIPE_CELL_STREAMS``), an int = that many
    (2 or more), ``False`` / 0 / 1 = one stream."""
    count = DEFAULT_CELL_STREAMS if enabled is True else int(enabled)
    for m in model.modules():
        if isinstance(m, Cell):
            m.streams = count if count >= 2 else 0


def amoebanetd(num_classes: int = 10, num_layers: int = 4, num_filters: int = 512
               ) -> nn.Sequential:
    """Build AmoebaNet-D(num_layers, num_filters) as a flat ``nn.Sequential``."""
    assert num_layers % 3 == 0
    repeat = num_layers // 3
    channels = num_filters // 4
    state = {'pp': channels, 'p': channels, 'c': channels, 'red_prev': False}

    def cells(reduction: bool, scale: int, count: int) -> Iterator[Cell]:
        state['c'] *= scale
        for _ in range(count):
            cell = Cell(state['pp'], state['p'], state['c'], reduction, state['red_prev'])
            state['pp'] = state['p']
            state['p'] = state['c'] * len(cell.concat)
            state['red_prev'] = reduction
            yield cell

    layers: 'OrderedDict[str, nn.Module]' = OrderedDict()
    layers['stem1'] = Stem(channels)
    layers['stem2'] = next(cells(True, 2, 1))
    layers['stem3'] = next(cells(True, 2, 1))
    for i, cell in enumerate(cells(False, 1, repeat)):
        layers[f'cell1_normal{i + 1}'] = cell
    layers['cell2_reduction'] = next(cells(True, 2, 1))
    for i, cell in enumerate(cells(False, 1, repeat)):
        layers[f'cell3_normal{i + 1}'] = cell
    layers['cell4_reduction'] = next(cells(True, 2, 1))
    for i, cell in enumerate(cells(False, 1, repeat)):
        layers[f'cell5_normal{i + 1}'] = cell
    layers['classify'] = Classify(state['p'], num_classes)
    return nn.Sequential(layers)
