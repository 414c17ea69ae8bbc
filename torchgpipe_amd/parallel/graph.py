"""Whole-step hipGraph capture of a one-rank pipeline stage.

A GPipe step launches one kernel sequence per layer, micro-batch and pass from Python.
For AmoebaNet-D(18, 256) at 32 micro-batches that is ~110 k launches per step whose host
cost alone is ~1.45 s (``benchmarks/stage_harness.py`` with 1-image micro-batches, where the
device idles: ``profiles/r2/host_cost_amoeba.md``), against 2.04 s of kernels at the
benchmark's 20-image micro-batches -- the host is one kernel-speed-up away from being the
bottleneck.  :class:`StepGraph` records the whole training step -- every micro-batch's
forward, recomputation and backward, and optionally the optimizer step -- into one
``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) after a few eager warm-up steps, then runs
each later step as a single graph launch: the same kernels, in the same order, with no
Python, autograd or dispatcher work per launch.

There is no tracing compiler involved: capture records the HIP launches of the eager step
(``hipStreamBeginCapture``), so what runs is exactly the eager program.

Requirements, checked up front:

* one rank (``world == 1``): point-to-point traffic is not captured;
* static shapes and addresses: ``input`` / ``target`` are copied into static buffers
  before each replay (skipped when the caller passes the static buffers themselves);
* no random ops: replaying a graph re-issues the captured Philox ``(seed, offset)``
  pairs, so dropout masks would repeat every step.  Partitions with dropout modules
  (``p > 0``) are refused, and framework RNG ops raise if they draw inside a capture
  (:func:`torchgpipe_amd.utils.rng.philox_pair`).

Each replay computes the step's gradients from scratch (the first micro-batch writes
``param.grad``, later ones accumulate), i.e. the eager step that follows
``optimizer.zero_grad()``; ``param.grad`` holds them after the replay.

What a replay does not see, and how it is handled:

* ``.grad`` ownership: the gradients live in the graph's memory pool.  Replays write
  those tensors whatever ``param.grad`` points to, so :meth:`StepGraph.step` re-attaches
  them before each replay (a ``zero_grad(set_to_none=True)`` in between is harmless).
* Optimizer hyperparameters are baked into the captured kernels as constants: an LR
  scheduler or a change to ``param_groups`` after the capture would be silently ignored.
  The scalar hyperparameters are snapshotted at capture and every replay checks them;
  a change raises instead of training with stale values (re-create the StepGraph, or use
  an optimizer built with ``capturable=True`` and tensor hyperparameters).

Shapes first met inside the capture would run the implicit-GEMM kernels' heuristic plans,
which is why the warm-up steps (which autotune them) come first.
"""
from typing import Callable, Dict, List, Optional, Tuple

import torch
from torch import Tensor, nn

from torchgpipe_amd.parallel.stage import PipelineStage
from torchgpipe_amd.utils.bigstack import call_with_big_stack

__all__ = ['StepGraph', 'rng_modules']


def rng_modules(module: nn.Module) -> List[str]:
    """Names of the sub-modules of ``module`` that draw random numbers in training mode."""
    found = []
    for name, m in module.named_modules():
        p = getattr(m, 'p', None)
        if 'Drop' in type(m).__name__ and isinstance(p, (int, float)) and p > 0:
            found.append(name or type(m).__name__)
    return found


class StepGraph:
    """Capture ``stage.train_step`` (+ ``optimizer.step()``) once; replay it per step.

    Args:
        stage: a one-rank :class:`~torchgpipe_amd.parallel.PipelineStage` on a GPU.
        loss_fn: ``loss_fn(output, target)``, as for ``PipelineStage.train_step``.
        optimizer: stepped inside the graph when given (its update is captured too).
        warmup: eager steps before the capture (allocator pools, autotuned convolution
            plans, optimizer state, lazily initialised libraries).

    ``step(input, target)`` returns the step's loss tensor, which the next replay
    overwrites.  On a CPU stage every step runs eagerly (there is nothing to capture).
    """

    def __init__(self, stage: PipelineStage, loss_fn: Callable[[Tensor, Tensor], Tensor],
                 optimizer: Optional[torch.optim.Optimizer] = None, *,
                 warmup: int = 2) -> None:
        if stage.world != 1:
            raise ValueError('StepGraph captures one-rank stages only (the graph cannot '
                             'hold point-to-point transfers)')
        rng = rng_modules(stage.partition)
        if rng:
            raise ValueError('StepGraph: the partition draws random numbers, which a graph '
                             f'replay would repeat every step: {", ".join(rng[:4])}'
                             f'{" ..." if len(rng) > 4 else ""}')
        if warmup < 1:
            raise ValueError('StepGraph needs at least one eager warm-up step')
        self.stage = stage
        self.loss_fn = loss_fn
        self.optimizer = optimizer
        self.warmup = warmup
        self._warm = 0
        self._graph: Optional[torch.cuda.CUDAGraph] = None
        self._input: Optional[Tensor] = None
        self._target: Optional[Tensor] = None
        self._loss: Optional[Tensor] = None
        self._grads: List[Tuple[Tensor, Tensor]] = []
        self._hyper: List[Dict[str, object]] = []

    @property
    def captured(self) -> bool:
        return self._graph is not None

    @property
    def static_input(self) -> Optional[Tensor]:
        """The buffer replays read the input from (``None`` before the capture)."""
        return self._input

    @property
    def static_target(self) -> Optional[Tensor]:
        return self._target

    def _zero_grad(self) -> None:
        if self.optimizer is not None:
            self.optimizer.zero_grad(set_to_none=True)
        else:
            for p in self.stage.parameters():
                p.grad = None

    def _eager(self, input: Tensor, target: Tensor) -> Tensor:
        loss = self.stage.train_step(input, target, self.loss_fn)
        assert loss is not None
        if self.optimizer is not None:
            self.optimizer.step()
        return loss

    def step(self, input: Tensor, target: Tensor) -> Tensor:
        """One training step: eager during warm-up, then capture, then graph replays."""
        device = self.stage.device
        if device.type != 'cuda':
            self._zero_grad()
            return self._eager(input, target)
        if self._graph is None and self._warm < self.warmup:
            # Warm-up on a side stream, as graph capture requires of everything it will
            # record (lazy initialisations must not happen inside the capture) -- and on
            # the big-stack thread that will capture and replay: its library handles
            # (hipBLASLt, MIOpen) are created here, outside the capture.
            self._zero_grad()
            side = torch.cuda.Stream(device)
            side.wait_stream(torch.cuda.current_stream(device))
            with torch.cuda.stream(side):
                loss = call_with_big_stack(lambda: self._eager(input, target))
            torch.cuda.current_stream(device).wait_stream(side)
            self._warm += 1
            return loss
        if self._graph is None:
            # captured on the big-stack thread too: ending the capture of a multi-stream
            # step (three-stream AmoebaNet cells) walks the DAG recursively as well and
            # overflowed the 8 MiB main-thread stack (utils/bigstack.py)
            call_with_big_stack(lambda: self._capture(input, target))
        assert self._graph is not None and self._input is not None and self._target is not None
        if self._hyperparameters() != self._hyper:
            raise RuntimeError('StepGraph: optimizer hyperparameters changed since the capture '
                               '(the replay would keep the captured values); re-create the '
                               'StepGraph or use a capturable optimizer with tensor '
                               'hyperparameters')
        for param, grad in self._grads:
            if param.grad is not grad:
                param.grad = grad
        if input is not self._input:
            self._input.copy_(input)
        if target is not self._target:
            self._target.copy_(target)
        # replays from a big-stack thread: the runtime walks a multi-stream graph
        # recursively when it launches it (utils/bigstack.py)
        call_with_big_stack(self._graph.replay)
        assert self._loss is not None
        return self._loss

    __call__ = step

    def _capture(self, input: Tensor, target: Tensor) -> None:
        device = self.stage.device
        self._input = input.detach().clone()
        self._target = target.detach().clone()
        # Gradients are created inside the capture (from the graph's memory pool) and
        # rewritten by every replay.
        self._zero_grad()
        # the capture stream and the side streams multi-stream cells pair with it exist
        # before the capture starts (no stream creation inside it)
        capture = torch.cuda.Stream(device)
        from torchgpipe_amd.models.amoebanet import prepare_side_streams
        prepare_side_streams(device, capture)
        torch.cuda.synchronize(device)
        graph = torch.cuda.CUDAGraph()
        self._hyper = self._hyperparameters()
        from torchgpipe_amd.models.amoebanet import whole_step_capture
        with torch.cuda.graph(graph, stream=capture), whole_step_capture():
            self._loss = self._eager(self._input, self._target)
        self._graph = graph
        self._grads = [(p, p.grad) for p in self.stage.parameters() if p.grad is not None]

    def _hyperparameters(self) -> List[Dict[str, object]]:
        """The optimizer's scalar hyperparameters, per parameter group."""
        if self.optimizer is None:
            return []
        return [{k: v for k, v in group.items()
                 if k != 'params' and isinstance(v, (int, float, bool, tuple, str, type(None)))}
                for group in self.optimizer.param_groups]
