"""Automatic balancing of a sequential module across pipeline partitions.

Parity: ``torchgpipe/balance/__init__.py:33-156``::

    from torchgpipe_amd import GPipe
    from torchgpipe_amd.balance import balance_by_time

    sample = torch.empty(128, 3, 224, 224)
    balance = balance_by_time(torch.cuda.device_count(), model, sample)
    gpipe = GPipe(model, balance, chunks=8)

The partition itself is solved exactly (min-max block cost, then most even;
see :mod:`.blockpartition`), not with the reference's heuristic.
"""
from typing import List, Tuple, Union

import torch
from torch import Tensor, nn

from torchgpipe_amd.balance import blockpartition
from torchgpipe_amd.balance.profile import profile_sizes, profile_times

__all__ = ['balance_by_time', 'balance_by_size', 'balance_cost']

Device = Union[torch.device, int, str]
Tensors = Tuple[Tensor, ...]
TensorOrTensors = Union[Tensor, Tensors]


def balance_cost(cost: List[int], partitions: int) -> List[int]:
    return blockpartition.solve_splits(cost, partitions)


def balance_by_time(partitions: int, module: nn.Sequential, sample: TensorOrTensors, *,
                    timeout: float = 1.0, device: Device = torch.device('cuda')) -> List[int]:
    """Balance by measured forward+backward time per layer.

    Args:
        partitions: number of partitions.
        module: the ``nn.Sequential`` to split.
        sample: example input (any batch size; a micro-batch-sized one is best).
        timeout: profile for at least this many seconds.
        device: ``'cpu'`` or a GPU on which each layer is profiled.
    """
    times = profile_times(module, sample, timeout, torch.device(device))
    return balance_cost(times, partitions)


def balance_by_size(partitions: int, module: nn.Sequential, input: TensorOrTensors, *,
                    chunks: int = 1, param_scale: float = 2.0,
                    device: Device = torch.device('cuda')) -> List[int]:
    """Balance by activation + parameter memory per layer.

    ``param_scale`` counts parameter copies for training (gradient + optimizer
    state): SGD 2–3, Adam 4–5, Adadelta 4, Adagrad 3, RMSprop 3–5.
    """
    sizes = profile_sizes(module, input, chunks, param_scale, torch.device(device))
    return balance_cost(sizes, partitions)
