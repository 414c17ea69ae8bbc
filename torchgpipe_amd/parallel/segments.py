"""Per-cell hipGraph replay for multi-rank pipeline stages ("segments").

A multi-rank stage cannot be captured as one graph the way :class:`StepGraph` captures a
one-rank step: its point-to-point transfers sit between the cells, and a rank must post
them as soon as the data exists.  What *can* be captured is each cell's compute -- the
part that costs the host its time (AmoebaNet-D(18,256) n8m32 stages spend 85-98 % of
their device time enqueueing launches, ``profiles/r3/stage_harness_amoeba_n8m32_ref.json``).
With ``PipelineStage(graph_cells=True)`` every *checkpointed* micro-batch ``i`` of the
stage becomes three graphs:

* ``F_i`` -- the no-grad forward: persistent input buffers -> static outputs;
* ``R_i`` -- the recomputation: the same inputs, now as autograd leaves, with grad;
* ``B_i`` -- the backward through ``R_i``'s graph: static output-gradient buffers ->
  input gradients (static) plus the parameter gradients, accumulated into ``.grad``;

and every non-checkpointed one (``except_last``'s last micro-batch, ``never``) two: ``F_i``
captured *with* grad (its saved activations live in the graph's memory pool) and ``B_i``.

The RCCL sends and receives stay eager, between the graph launches, exactly where the
eager schedule posts them (``parallel/stage.py``), and the launches go to the same lanes
the eager schedule uses (forward lanes, recompute lanes), so the overlap structure is
unchanged.  This is the reference's per-cell split (``torchgpipe/checkpoint.py:234-308``:
``Checkpoint`` / ``Recompute``, and ``torchgpipe/pipeline.py:144-249``) with each part
replayed instead of re-traced.  Outputs reach the loss (last stage) or the sends as
detached leaves, so no autograd graph outside the captures ever links to a parameter:
each capture creates its own ``AccumulateGrad`` nodes on its own capture stream.

How static addresses are kept without copies:

* received activations, skips and gradients land in persistent receive buffers
  (``P2P.recv(..., persistent=True)``), one per (message, micro-batch), which the graphs
  read in place; the first stage copies its micro-batch into a persistent input buffer;
* derived weights (Winograd transforms, transposes, grouped-GEMM concatenations) are
  refreshed *in place* at the start of every step (``ops.conv.refresh_step_caches``);
* parameter gradients are allocated before the capture; the replays accumulate into them.
  At the start of a step a buffer is zeroed only when the user released the gradient
  (``zero_grad(set_to_none=True)``: ``.grad`` is None) -- a ``.grad`` still attached keeps
  its value and the step adds to it, as eager autograd does (gradient accumulation over
  several ``train_step`` calls); a ``.grad`` the user replaced is copied into the buffer
  first.  Parameters that no captured backward reaches keep ``.grad`` None, as in eager
  mode (an optimizer then skips them);
* dropout reads a device-resident Philox state per cell (``utils.rng.PhiloxSlot``) that
  the host fills with freshly reserved ``(seed, offset)`` values before the step's replays,
  so masks change every step and ``F_i`` / ``R_i`` agree bit for bit.

Life cycle: ``warmup`` eager steps (library handles, tuned kernel plans, slab and cache
allocation, message metadata), one capture step (each graph is captured and immediately
replayed, without overlap), then replays.  A new input signature, ``eval()`` or
``no_grad`` falls back to eager steps (a new signature re-captures).

Memory: two private graph pools; cell ``i`` uses pool ``(m - 1 - i) % 2`` for all of its
graphs.  Cells that run concurrently -- neighbours on the two forward lanes, or a backward
beside the next cell's recomputation on the two recompute lanes -- are always in different
pools, and the graphs of one pool replay in their capture order (forward phase, then
backward phase), so no graph ever reads scratch another one is writing.
"""
import contextlib
import time
from typing import Any, Callable, Iterator, List, Optional, Sequence, Tuple

import torch
from torch import Tensor, nn

from torchgpipe_amd.checkpoint import enable_checkpointing, enable_recomputing
from torchgpipe_amd.ops import gradacc
from torchgpipe_amd.utils import rng

__all__ = ['Segments', 'SegmentCell']

Tensors = Tuple[Tensor, ...]


@contextlib.contextmanager
def _capturing(graph: 'torch.cuda.CUDAGraph', stream: 'torch.cuda.Stream',
               pool: Any) -> Iterator[None]:
    """Capture onto ``graph`` from ``stream`` into the private memory ``pool``.

    ``thread_local`` capture mode: other threads (RCCL proxies, the process group's
    watchdog, the autograd engine's device thread) may keep making CUDA calls.  Unlike
    ``torch.cuda.graph`` this neither synchronises the device nor empties the cache: a
    device-wide sync could wait on a receive whose sender is itself waiting on this rank.
    """
    with torch.cuda.stream(stream):
        graph.capture_begin(pool=pool, capture_error_mode='thread_local')
        try:
            yield
        finally:
            graph.capture_end()


class SegmentCell:
    """The captured graphs and static tensors of one checkpointed micro-batch."""

    __slots__ = ('index', 'checkpointed', 'fwd', 'rec', 'bwd', 'inputs', 'outputs', 'out_atomic',
                 'n_act_out', 'leaves', 'rec_out', 'gouts', 'gins', 'slot', 'increment',
                 'user_out', 'recomputed', 'out_grad')

    def __init__(self, index: int, checkpointed: bool, slot: Optional[rng.PhiloxSlot]) -> None:
        self.index = index
        self.checkpointed = checkpointed    # F without grad + R, else F with grad
        self.fwd: Optional[torch.cuda.CUDAGraph] = None
        self.rec: Optional[torch.cuda.CUDAGraph] = None
        self.bwd: Optional[torch.cuda.CUDAGraph] = None
        self.inputs: List[Tensor] = []      # what F_i / R_i read (persistent)
        self.outputs: List[Tensor] = []     # F_i's static outputs
        self.out_atomic = True
        self.n_act_out = 0
        self.leaves: List[Tensor] = []      # R_i's autograd leaves (views of inputs)
        self.rec_out: List[Tensor] = []     # R_i's outputs (graph kept for the B capture)
        self.gouts: List[Optional[Tensor]] = []  # B_i's output-gradient buffers
        self.gins: List[Tensor] = []        # B_i's input gradients (static)
        self.slot = slot
        self.increment = 0                  # Philox counters one pass of the cell draws
        self.user_out: List[Tensor] = []    # last stage: output leaves handed to the loss
        self.recomputed = False             # R_i replayed in this step
        self.out_grad: List[bool] = []      # which outputs require grad


class Segments:
    """Captured cells of one :class:`~torchgpipe_amd.parallel.PipelineStage` for one
    input signature.

    Args:
        partition: the stage's module (parameters, step caches).
        device: the stage's GPU.
        cells: number of micro-batches (each gets its graphs).
        stop: the first ``stop`` micro-batches are checkpointed.
        warmup: eager steps before the capture step.
    """

    def __init__(self, partition: nn.Module, device: torch.device, cells: int, stop: int,
                 warmup: int = 1) -> None:
        self.partition = partition
        self.device = device
        self.warmup = warmup
        self.steps = 0
        self.captured = False
        self.pools = [torch.cuda.graph_pool_handle(), torch.cuda.graph_pool_handle()]
        # (fresh per instance, not named: a stage's captures must not share their streams
        # -- and the cell side streams keyed on them -- with another stage's graphs in the
        # same process)
        self.streams = [torch.cuda.Stream(device), torch.cuda.Stream(device)]
        from torchgpipe_amd.models.amoebanet import prepare_side_streams
        for s in self.streams:  # cell side streams paired with the capture streams
            prepare_side_streams(device, s)
        self.slots = torch.zeros(cells, 2, dtype=torch.int64, device=device)
        self.cells = [SegmentCell(i, i < stop, rng.PhiloxSlot(self.slots[i]))
                      for i in range(cells)]
        self.grads: List[Tuple[Tensor, Tensor]] = []
        self.used: set = set()  # ids of the parameters the captured backwards reach
        self.pending: List[Any] = []
        self._zeros: List[Tensor] = []
        # host seconds spent inside graph launches (hipGraphLaunch enqueues every node;
        # it blocks when the hardware queue is full, i.e. when the GPU is the bottleneck)
        self.launch_s = 0.0

    # -- step ---------------------------------------------------------------------------------

    @property
    def phase(self) -> str:
        """``'eager'`` (warm-up), ``'capture'`` or ``'replay'`` for the current step."""
        if self.captured:
            return 'replay'
        return 'capture' if self.steps > self.warmup else 'eager'

    def begin_step(self) -> str:
        """Start a step: returns its phase.  Capture / replay steps attach the static
        gradient buffers -- zeroed where the user released ``.grad``, holding the user's
        gradient otherwise, so the step accumulates like eager autograd -- and replays get
        fresh Philox values in every cell's slot."""
        self.steps += 1
        phase = self.phase
        if phase == 'capture':
            self.grads = []
            self.used = set()
            for p in self.partition.parameters():
                if not p.requires_grad:
                    continue
                g = torch.zeros_like(p, memory_format=torch.contiguous_format)
                if p.grad is not None:
                    g.copy_(p.grad)
                p.grad = g
                self.grads.append((p, g))
        elif phase == 'replay':
            zero = []
            for p, g in self.grads:
                if p.grad is None:
                    p.grad = g
                    zero.append(g)
                elif p.grad is not g:
                    g.copy_(p.grad)
                    p.grad = g
            if zero:
                torch._foreach_zero_(zero)
        if phase == 'replay':
            self._fill_slots(self.cells)
        return phase

    def _note_reached(self, outputs: Sequence[Tensor]) -> None:
        """Record the parameters the autograd graph of ``outputs`` reaches (their
        AccumulateGrad nodes), before a backward capture consumes that graph."""
        seen = set()
        todo = [t.grad_fn for t in outputs if t.grad_fn is not None]
        while todo:
            fn = todo.pop()
            if fn is None or fn in seen:
                continue
            seen.add(fn)
            var = getattr(fn, 'variable', None)
            if var is not None:
                self.used.add(id(var))
            todo.extend(nxt for nxt, _ in fn.next_functions if nxt is not None)

    def _fill_slots(self, cells: Sequence[SegmentCell]) -> None:
        """Reserve the cells' Philox counters from the device generator and write the
        ``(seed, base offset)`` of each into its slot (one pinned host-to-device copy)."""
        total = sum(c.increment for c in cells)
        if total == 0:
            return
        seed, base = rng.reserve(self.device, total)
        seed = seed - (1 << 64) if seed >= (1 << 63) else seed
        vals = torch.empty(len(cells), 2, dtype=torch.int64, pin_memory=True)
        for k, c in enumerate(cells):
            vals[k, 0] = seed
            vals[k, 1] = base
            base += c.increment
        first = cells[0].index
        self.slots[first:first + len(cells)].copy_(vals, non_blocking=True)

    # -- forward ------------------------------------------------------------------------------

    def static_inputs(self, i: int, flat: Sequence[Tensor]) -> List[Tensor]:
        """``flat`` at the addresses ``F_i`` / ``R_i`` read: the received persistent buffers
        themselves, else (first stage, host-staged receives) copies into the cell's own."""
        cell = self.cells[i]
        if not cell.inputs:
            return list(flat)
        for dst, src in zip(cell.inputs, flat):
            if dst.data_ptr() != src.data_ptr():
                dst.copy_(src)
        return cell.inputs

    def adopt_inputs(self, i: int, flat: Sequence[Tensor], owned: bool) -> List[Tensor]:
        """Fix cell ``i``'s input buffers at capture: ``flat`` itself when it is persistent
        (``owned`` False: received buffers), else copies the cell keeps."""
        cell = self.cells[i]
        # (requires_grad as received: it decides which input gradients the cell returns)
        if owned:
            cell.inputs = [t.detach().clone().requires_grad_(t.requires_grad) for t in flat]
        else:
            cell.inputs = [t.detach().requires_grad_(t.requires_grad) for t in flat]
        return cell.inputs

    def pool_index(self, i: int) -> int:
        """Memory pool and capture stream of cell ``i`` (see the module docstring)."""
        return (len(self.cells) - 1 - i) % 2

    def forward(self, i: int, fn: Callable[[Tensors], Tensors],
                lane: 'torch.cuda.Stream') -> List[Tensor]:
        """Run (capture, or replay) cell ``i``'s forward on ``lane`` -- without grad for a
        checkpointed cell, with grad otherwise; returns its static outputs."""
        cell = self.cells[i]
        if cell.fwd is None:
            k = self.pool_index(i)
            graph = torch.cuda.CUDAGraph()
            assert cell.slot is not None
            if cell.checkpointed:
                with _capturing(graph, self.streams[k], self.pools[k]), torch.no_grad(), \
                        enable_checkpointing(), rng.slot_scope(cell.slot):
                    out = list(fn(tuple(cell.inputs)))
                # as the outputs of an eager Checkpoint node: every float output
                cell.out_grad = [t.is_floating_point() for t in out]
            else:
                cell.leaves = [t.detach().requires_grad_(t.requires_grad) for t in cell.inputs]
                with _capturing(graph, self.streams[k], self.pools[k]), torch.enable_grad(), \
                        rng.slot_scope(cell.slot):
                    cell.rec_out = list(fn(tuple(cell.leaves)))
                out = [t.detach() for t in cell.rec_out]
                cell.out_grad = [t.requires_grad for t in cell.rec_out]
            cell.increment = cell.slot.delta
            cell.outputs = out
            cell.fwd = graph
            self._fill_slots([cell])
        lane.wait_stream(torch.cuda.current_stream(self.device))
        self._replay(cell.fwd, lane)
        return cell.outputs

    def user_outputs(self, i: int) -> List[Tensor]:
        """The static outputs as fresh autograd leaves, requiring grad where the eager cell's
        outputs do (the message metadata of the eager warm-up says so, and the last stage's
        loss back-propagates into them)."""
        cell = self.cells[i]
        cell.user_out = [t.detach().requires_grad_(g) for t, g in zip(cell.outputs, cell.out_grad)]
        return cell.user_out

    # -- backward -----------------------------------------------------------------------------

    def recompute(self, i: int, fn: Optional[Callable[[Tensors], Tensors]],
                  lane: 'torch.cuda.Stream') -> None:
        """Run (capture, or replay) cell ``i``'s recomputation on ``lane`` (once per step;
        nothing for a non-checkpointed cell)."""
        cell = self.cells[i]
        if cell.recomputed or not cell.checkpointed:
            return
        k = self.pool_index(i)
        if cell.rec is None:
            assert fn is not None
            graph = torch.cuda.CUDAGraph()
            cell.leaves = [t.detach().requires_grad_(t.requires_grad) for t in cell.inputs]
            assert cell.slot is not None
            with _capturing(graph, self.streams[k], self.pools[k]), torch.enable_grad(), \
                    enable_recomputing(), rng.slot_scope(cell.slot):
                cell.rec_out = list(fn(tuple(cell.leaves)))
            if cell.slot.delta != cell.increment:
                raise RuntimeError(f'cell {i}: the recomputation drew {cell.slot.delta} Philox '
                                   f'counters, the forward {cell.increment}')
            cell.rec = graph
        lane.wait_stream(torch.cuda.current_stream(self.device))
        self._replay(cell.rec, lane)
        cell.recomputed = True

    def backward(self, i: int, grads: Sequence[Optional[Tensor]], persistent: Sequence[bool],
                 lane: 'torch.cuda.Stream') -> List[Tensor]:
        """Run (capture, or replay) cell ``i``'s backward on ``lane`` (ordered by the caller):
        ``grads[n]`` is the gradient of output ``n`` (``None``: none), ``persistent[n]``
        whether it sits in a persistent receive buffer (used in place; other gradients,
        e.g. the last stage's loss gradients, are copied into buffers of the cell's own).
        Returns the input gradients (static tensors; zeros for inputs that get none)."""
        cell = self.cells[i]
        if cell.bwd is None:
            k = self.pool_index(i)
            cell.gouts = []
            for y, g, keep in zip(cell.rec_out, grads, persistent):
                if g is None or not y.requires_grad:
                    cell.gouts.append(None)
                else:
                    cell.gouts.append(g.detach() if keep else g.detach().clone())
            pairs = [(y, g) for y, g in zip(cell.rec_out, cell.gouts) if g is not None]
            self._note_reached([p[0] for p in pairs])
            graph = torch.cuda.CUDAGraph()
            with _capturing(graph, self.streams[k], self.pools[k]):
                if pairs:
                    torch.autograd.backward([p[0] for p in pairs], [p[1] for p in pairs])
            cell.rec_out = []  # the recomputed graph was consumed by the capture
            gins = []
            for leaf in cell.leaves:
                if leaf.grad is None:
                    zero = torch.zeros_like(leaf)
                    self._zeros.append(zero)
                    gins.append(zero)
                else:
                    gins.append(leaf.grad)
            cell.gins = gins
            cell.bwd = graph
        else:
            for dst, g in zip(cell.gouts, grads):
                if dst is not None and g is not None and dst.data_ptr() != g.data_ptr():
                    dst.copy_(g)
        lane.wait_stream(torch.cuda.current_stream(self.device))
        self._replay(cell.bwd, lane)
        cell.recomputed = False
        return cell.gins

    def _replay(self, graph: 'torch.cuda.CUDAGraph', lane: 'torch.cuda.Stream') -> None:
        t0 = time.perf_counter()
        with torch.cuda.stream(lane):
            graph.replay()
        self.launch_s += time.perf_counter() - t0

    def end_backward(self) -> None:
        """End of the step's backward (inside the deferral scope): the capture step records
        the weight-gradient slabs its graphs write; replay steps re-register them."""
        if not self.captured and self.phase == 'capture':
            self.pending = gradacc.pending_snapshot(self.device)
            self.captured = all(c.bwd is not None for c in self.cells)
            if self.captured:
                # parameters no captured backward reaches get no gradient, as in eager mode
                # (their buffers held the user's gradient or zeros: give the former back)
                keep = []
                for p, g in self.grads:
                    if id(p) in self.used:
                        keep.append((p, g))
                    elif p.grad is g:
                        p.grad = None if not bool(g.any()) else g
                self.grads = keep
        elif self.captured:
            gradacc.register_pending(self.device, self.pending)
        for c in self.cells:
            c.recomputed = False
