"""Per-layer profilers used by the automatic balancers.

Parity: ``torchgpipe/balance/profile.py:21-118``.

* :func:`profile_times` — forward + backward time per layer, on a deep copy of
  each layer (the user's module is never touched).  On GPUs each layer is
  timed with HIP events recorded on the current stream (device time, not host
  time), repeated until ``timeout`` seconds have elapsed.
* :func:`profile_sizes` — activation bytes per sample (allocator delta of a
  1-sample forward) × micro-batch size + parameter bytes × ``param_scale``.
"""
import copy
import time
from typing import Iterator, List, Tuple, Union

import torch
from torch import Tensor, nn

from torchgpipe_amd.microbatch import Batch

__all__: List[str] = []

Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]


def layerwise_sandbox(module: nn.Sequential, device: torch.device) -> Iterator[nn.Module]:
    """Yield a training-mode deep copy of each layer on ``device``."""
    for layer in module:
        clone = copy.deepcopy(layer)
        clone.to(device)
        clone.train()
        yield clone


def detach(batch: Batch) -> None:
    for i, x in enumerate(batch):
        batch[i] = x.detach().requires_grad_(x.requires_grad)


def _backward(batch: Batch) -> None:
    outputs = tuple(y for y in batch if y.requires_grad)
    if outputs:
        torch.autograd.backward(outputs, outputs)


def profile_times(module: nn.Sequential, sample: TensorOrTensors, timeout: float,
                  device: torch.device) -> List[int]:
    """Microseconds spent per layer (forward + backward), summed over iterations."""
    if any(p.grad is not None for p in module.parameters()):
        raise ValueError('some parameter already has gradient')

    base = Batch(sample)
    for i, x in enumerate(base):
        base[i] = x.detach().to(device).requires_grad_(x.requires_grad)

    layers = list(layerwise_sandbox(module, device))
    totals = [0.0 for _ in layers]
    on_gpu = device.type == 'cuda'
    start = time.time()
    while time.time() - start < timeout:
        batch = base
        for i, layer in enumerate(layers):
            detach(batch)
            if on_gpu:
                begin_ev = torch.cuda.Event(enable_timing=True)
                end_ev = torch.cuda.Event(enable_timing=True)
                begin_ev.record()
                batch = batch.call(layer)
                _backward(batch)
                end_ev.record()
                end_ev.synchronize()
                totals[i] += begin_ev.elapsed_time(end_ev) * 1e3
            else:
                tick = time.time()
                batch = batch.call(layer)
                _backward(batch)
                totals[i] += (time.time() - tick) * 1e6
    return [int(t) for t in totals]


def profile_sizes(module: nn.Sequential, input: TensorOrTensors, chunks: int,
                  param_scale: float, device: torch.device) -> List[int]:
    """Bytes per layer: activations of one micro-batch + scaled parameter bytes."""
    if device.type != 'cuda':
        raise ValueError('size profiler supports only CUDA device')

    batch = Batch(input)
    latent_scale = batch[0].size(0) / chunks
    for i, x in enumerate(batch):
        batch[i] = x[:1].detach().to(device).requires_grad_(x.requires_grad)

    layers = list(layerwise_sandbox(module, device))

    # Warm-up pass: the first GEMM/conv on a device lazily allocates library
    # workspaces (hipBLASLt, MIOpen) through the caching allocator, which would
    # otherwise be billed to whichever layer happens to run first.
    warm = Batch(tuple(batch)) if not batch.atomic else Batch(batch.tensor)
    with torch.no_grad():
        for layer in layers:
            warm = warm.call(layer)
    del warm

    sizes: List[int] = []
    for layer in layers:
        detach(batch)
        before = torch.cuda.memory_allocated(device)
        batch = batch.call(layer)
        after = torch.cuda.memory_allocated(device)
        params = sum(p.numel() * p.element_size() for p in layer.parameters())
        sizes.append(int((after - before) * latent_scale + params * param_scale))
    return sizes
