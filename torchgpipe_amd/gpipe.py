"""The ``GPipe`` module: single-process, multi-device pipeline parallelism (layer L7).

Parity: ``torchgpipe/gpipe.py:34-380``.  Public contract kept verbatim:

* ``GPipe(module: nn.Sequential, balance, *, devices=None, chunks=1,
  checkpoint='except_last', deferred_batch_norm=False)``
* Sequential-like ``len`` / indexing / iteration over the wrapped layers,
  attributes ``balance``, ``devices``, ``chunks``, ``checkpoint``,
  ``partitions``; ``cuda()``/``cpu()``/``to(device)`` are denied (placement
  is managed), ``to(dtype)`` is allowed.
* State-dict keys ``partitions.<j>.<child-name>.<param>``.

MI355X-specific design:

* Copy streams come from a small per-device :class:`StreamPool` instead of
  ``chunks`` streams per device, and the device threads are persistent
  (:class:`~torchgpipe_amd.worker.WorkerPool`).
* Peer access between the partition GPUs is enabled up front so that
  activation / gradient / skip hand-offs are direct xGMI copies.
"""
from collections import OrderedDict
from typing import Any, Iterable, Iterator, List, Optional, Tuple, Union, cast

import torch
from torch import Tensor, nn

from torchgpipe_amd import microbatch
from torchgpipe_amd.batchnorm import DeferredBatchNorm, set_micro_batches
from torchgpipe_amd.ops.conv import new_step as wino_new_step
from torchgpipe_amd.ops.dropout import convert_dropout
from torchgpipe_amd.ops.fusion import relink
from torchgpipe_amd.pipeline import Pipeline
from torchgpipe_amd.skip.layout import inspect_skip_layout
from torchgpipe_amd.skip.skippable import verify_skippables
from torchgpipe_amd.stream import AbstractStream, StreamPool, current_stream, named_stream
from torchgpipe_amd.utils.meta import is_meta, materialize
from torchgpipe_amd.worker import WorkerPool

__all__ = ['GPipe', 'BalanceError', 'verify_module', 'split_module']

Device = Union[torch.device, int, str]
Devices = Union[Iterable[Device], List[Device]]
Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]


def recommend_auto_balance(message: str) -> str:
    """Append a pointer to :mod:`torchgpipe_amd.balance` to an error message."""
    return f'''{message}

If your model is still under development, its optimal balance would change
frequently. In this case, we highly recommend 'torchgpipe_amd.balance' (the
equivalent of 'torchgpipe.balance') for naive automatic balancing:

  from torchgpipe_amd import GPipe
  from torchgpipe_amd.balance import balance_by_time

  partitions = torch.cuda.device_count()
  sample = torch.empty(...)
  balance = balance_by_time(partitions, model, sample)

  model = GPipe(model, balance, ...)
'''


def verify_module(module: nn.Sequential) -> None:
    if not isinstance(module, nn.Sequential):
        raise TypeError('module must be nn.Sequential to be partitioned')
    if len(list(module.named_children())) != len(module):
        raise ValueError('module with duplicate children is not supported')
    total = len(list(module.parameters()))
    per_child = sum(len(list(child.parameters())) for child in module.children())
    if total != per_child:
        raise ValueError('module with duplicate parameters in distinct children is not supported')


class BalanceError(ValueError):
    pass


def check_balance(module: nn.Sequential, balance: List[int]) -> None:
    if len(module) != sum(balance):
        raise BalanceError('module and sum of balance have different length '
                           f'(module: {len(module)}, sum of balance: {sum(balance)})')
    if any(x <= 0 for x in balance):
        raise BalanceError(f'all balance numbers must be positive integer (balance: {balance})')


def partition_layers(module: nn.Sequential,
                     balance: List[int]) -> List['OrderedDict[str, nn.Module]']:
    """Group the named children of ``module`` into ``len(balance)`` chunks."""
    groups: List['OrderedDict[str, nn.Module]'] = []
    children = iter(module.named_children())
    for size in balance:
        group: 'OrderedDict[str, nn.Module]' = OrderedDict()
        for _ in range(size):
            name, layer = next(children)
            group[name] = layer
        groups.append(group)
    return groups


def split_module(module: nn.Sequential, balance: Iterable[int], devices: List[torch.device],
                 ) -> Tuple[List[nn.Sequential], List[int], List[torch.device]]:
    """Split ``module`` into per-device ``nn.Sequential`` partitions.

    Raises ``BalanceError`` for a wrong balance and ``IndexError`` when there
    are fewer devices than partitions.  Extra devices are dropped.
    """
    balance = list(balance)
    check_balance(module, balance)
    if len(balance) > len(devices):
        raise IndexError('too few devices to hold given partitions '
                         f'(devices: {len(devices)}, partitions: {len(balance)})')
    partitions = []
    for group, device in zip(partition_layers(module, balance), devices):
        partition = nn.Sequential(group)
        if is_meta(partition):
            # Built on the meta device: allocate + initialise on the target GPU.
            materialize(partition, device)
        else:
            partition.to(device)
        # Conv-BN(-ReLU) runs fuse only inside one partition (ops/fusion.py)
        relink(partition)
        partitions.append(partition)
    del devices[len(balance):]
    return cast(List[nn.Sequential], nn.ModuleList(partitions)), balance, devices


def enable_peer_access(devices: List[torch.device]) -> None:
    """Open peer access between every pair of partition GPUs (direct xGMI copies).

    PyTorch enables peer access lazily inside the first peer copy between two
    devices (``hipDeviceEnablePeerAccess``, a synchronising call).  Touching
    every pair once with a 1-element copy keeps that setup out of the first
    training step.  Skip routes can connect any two partitions, so all pairs
    are opened — the MI355X xGMI mesh is fully connected.
    """
    gpus = sorted({d.index for d in devices if d.type == 'cuda' and d.index is not None})
    for a in gpus:
        for b in gpus:
            if a != b and torch.cuda.can_device_access_peer(a, b):
                torch.zeros(1, device=torch.device('cuda', a)).to(torch.device('cuda', b))


MOVING_DENIED = TypeError('denied to move parameters and buffers, '
                          'because GPipe should manage device placement')


class _JoinLanes(torch.autograd.Function):
    """Identity on the pipeline's output whose backward (the first to run) schedules a
    callback for the end of the backward pass: the caller's streams then wait for the
    forward lanes.  The fused ops on the lanes add into ``.grad`` outside autograd
    (``ops/gradacc.py``), so the engine's own end-of-backward sync, which covers only the
    streams its ``AccumulateGrad`` nodes ran on, would let the optimizer read gradients the
    last micro-batch's backward is still adding to."""

    @staticmethod
    def forward(ctx, lanes: List[AbstractStream], *outputs: Tensor):  # type: ignore[override]
        ctx.lanes = lanes
        views = tuple(t.view_as(t) for t in outputs)
        frozen = [v for v, t in zip(views, outputs) if not t.requires_grad]
        if frozen:
            ctx.mark_non_differentiable(*frozen)
        return views if len(views) > 1 else views[0]

    @staticmethod
    def backward(ctx, *grads: Tensor):  # type: ignore[override]
        lanes = ctx.lanes

        def join() -> None:  # (runs with the caller's current streams current)
            for lane in lanes:
                cast(torch.cuda.Stream, current_stream(lane.device)).wait_stream(lane)

        torch.autograd.Variable._execution_engine.queue_callback(join)  # type: ignore
        return (None,) + grads


class GPipe(nn.Module):
    """Wrap an ``nn.Sequential`` to train it with GPipe pipeline parallelism.

    ::

        model = nn.Sequential(a, b, c, d)
        model = GPipe(model, balance=[1, 1, 1, 1], chunks=8)
        output = model(input)

    Args:
        module: the sequential module to parallelise.
        balance: number of layers in each partition.

    Keyword Args:
        devices: devices of the partitions (default: all visible GPUs).
        chunks: number of micro-batches (default 1).
        checkpoint: ``'always'``, ``'except_last'`` (default) or ``'never'``.
        deferred_batch_norm: accumulate BatchNorm running statistics over the
            whole mini-batch instead of per micro-batch (default ``False``).
        copy_streams_per_device: size of the per-device copy-stream ring.
        philox_dropout: run the module's ``nn.Dropout`` / ``nn.Dropout2d`` layers on
            explicit Philox pairs replayed from each checkpoint's RNG tape instead of
            forking and restoring the global generators during recomputation
            (``ops.dropout.convert_dropout``; default ``False``: the reference's
            behaviour, bitwise equal to the plain model under the same seed).
        overlap_forward: compute the forward micro-batches of every partition without
            running statistics (no BatchNorm buffers; e.g. U-Net) alternately on two
            streams of its GPU ("lanes", like ``PipelineStage(overlap_forward=True)``), so
            micro-batch ``i + 1`` can run beside micro-batch ``i`` where its input is ready:
            on the first partition, and on any partition slower than its upstream.
            Backward passes keep the reference's order (the ``depend`` edges, with the
            autograd engine's cross-stream syncs).  Default ``False``: one stream per
            device, as the reference.
    """

    balance: List[int] = []
    devices: List[torch.device] = []
    chunks: int = 1
    checkpoint: str = 'except_last'

    def __init__(self, module: nn.Sequential, balance: Optional[Iterable[int]] = None, *,
                 devices: Optional[Devices] = None, chunks: int = chunks,
                 checkpoint: str = checkpoint, deferred_batch_norm: bool = False,
                 copy_streams_per_device: int = 4, philox_dropout: bool = False,
                 overlap_forward: bool = False) -> None:
        super().__init__()
        chunks = int(chunks)
        checkpoint = str(checkpoint)

        if balance is None:
            raise ValueError(recommend_auto_balance('balance is required'))
        if chunks <= 0:
            raise ValueError('number of chunks must be positive integer')
        if checkpoint not in ('always', 'except_last', 'never'):
            raise ValueError("checkpoint is not one of 'always', 'except_last', or 'never'")

        verify_module(module)
        verify_skippables(module)

        self.chunks = chunks
        self.checkpoint = checkpoint

        if deferred_batch_norm:
            module = DeferredBatchNorm.convert_deferred_batch_norm(module, chunks)
        if philox_dropout:
            convert_dropout(module)

        if devices is None:
            devices = range(torch.cuda.device_count())
        device_list = [torch.device(d) for d in devices]

        try:
            self.partitions, self.balance, self.devices = split_module(
                module, balance, device_list)
        except BalanceError as exc:
            raise ValueError(recommend_auto_balance(str(exc)))

        self._peers_ready = False
        self._stream_pool = StreamPool(copy_streams_per_device)
        self._copy_streams: List[List[AbstractStream]] = []
        self._workers = WorkerPool()
        self._skip_layout = inspect_skip_layout(self.partitions)
        self._has_dbn = any(isinstance(m, DeferredBatchNorm) for m in self.modules())
        self.overlap_forward = overlap_forward
        self._lanes: Optional[List[Optional[List[AbstractStream]]]] = None

    # -- Sequential-like interface ------------------------------------------------------------

    def __len__(self) -> int:
        return sum(len(p) for p in self.partitions)

    def __getitem__(self, index: int) -> nn.Module:
        layers = list(self)
        try:
            return layers[index]
        except IndexError:
            raise IndexError

    def __iter__(self) -> Iterator[nn.Module]:  # type: ignore[override]
        for partition in self.partitions:
            yield from partition

    # -- placement is managed -----------------------------------------------------------------

    def cuda(self, device: Optional[Device] = None) -> 'GPipe':  # type: ignore[override]
        raise MOVING_DENIED

    def cpu(self) -> 'GPipe':  # type: ignore[override]
        raise MOVING_DENIED

    def to(self, *args: Any, **kwargs: Any) -> 'GPipe':  # type: ignore[override]
        if 'device' in kwargs or 'tensor' in kwargs:
            raise MOVING_DENIED
        if args and (isinstance(args[0], (torch.device, int, str)) or torch.is_tensor(args[0])):
            raise MOVING_DENIED
        return super().to(*args, **kwargs)

    # -- execution ----------------------------------------------------------------------------

    def _ensure_copy_streams(self) -> List[List[AbstractStream]]:
        if not self._copy_streams:
            self._copy_streams = self._stream_pool.grid(self.devices, self.chunks)
        return self._copy_streams

    def _forward_lanes(self) -> Optional[List[Optional[List[AbstractStream]]]]:
        """Two named streams per stateless GPU partition (``overlap_forward``)."""
        if not self.overlap_forward or torch.cuda.is_available() and \
                torch.cuda.is_current_stream_capturing():
            return None
        if self._lanes is None:
            lanes: List[Optional[List[AbstractStream]]] = []
            for j, (part, dev) in enumerate(zip(self.partitions, self.devices)):
                stateful = any(isinstance(m, nn.modules.batchnorm._BatchNorm)
                               and m.track_running_stats for m in part.modules())
                lanes.append(None if dev.type != 'cuda' or stateful else
                             [named_stream(dev, f'gpipe-lane{j}-{k}') for k in (0, 1)])
            self._lanes = lanes
        return self._lanes

    def checkpoint_stop(self) -> int:
        if not self.training:
            return 0
        return {'always': self.chunks, 'except_last': self.chunks - 1,
                'never': 0}[self.checkpoint]

    def forward(self, input: TensorOrTensors) -> TensorOrTensors:  # type: ignore[override]
        """Run the pipeline.  Input/output: a tensor or a tuple of tensors."""
        microbatch.check(input)
        if not self.devices:
            return input

        if not self._peers_ready:
            enable_peer_access(self.devices)
            self._peers_ready = True
        wino_new_step()  # weights may have changed since the last step (even via .data)
        batches = microbatch.scatter(input, self.chunks)
        if self._has_dbn:
            set_micro_batches(self, len(batches))
        copy_streams = self._ensure_copy_streams()
        # K11: outputs land in preallocated buffers on the last device's copy streams
        # while later micro-batches still compute (no torch.cat after the pipeline)
        gatherer = microbatch.Gatherer([b[0].shape[0] if b[0].dim() else 1 for b in batches],
                                       copy_streams[-1])
        lanes = self._forward_lanes()
        pipeline = Pipeline(batches, list(self.partitions), self.devices, copy_streams,
                            self._skip_layout, self.checkpoint_stop(),
                            queues=self._workers.queues(self.devices),
                            on_output=gatherer.put, lanes=lanes)
        pipeline.run()
        output = gatherer.result(batches)
        if lanes is not None:
            # (a fallback gather reads the last partition's outputs on the current stream)
            used = [stream for lane in lanes if lane is not None for stream in lane]
            for stream in used:
                current_stream(stream.device).wait_stream(stream)  # type: ignore
            if used and torch.is_grad_enabled():
                outs = (output,) if isinstance(output, Tensor) else tuple(output)
                if any(t.requires_grad for t in outs):
                    joined = _JoinLanes.apply(used, *outs)
                    output = joined if isinstance(output, Tensor) else \
                        (tuple(joined) if isinstance(joined, tuple) else (joined,))
        return output

    def __getstate__(self) -> Any:
        state = self.__dict__.copy()
        state['_workers'] = WorkerPool()
        state['_stream_pool'] = StreamPool(self._stream_pool.size)
        state['_copy_streams'] = []
        state['_lanes'] = None
        return state
