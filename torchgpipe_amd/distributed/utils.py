"""``to(device, value)``: move a tensor / tuple across devices keeping ``requires_grad``.

Parity: ``torchgpipe/distributed/utils.py:6-22`` (tolerates ``None`` entries).
"""
from typing import Optional, Tuple, Union

import torch
from torch import Tensor

TensorOrTensors = Union[Tensor, Tuple[Optional[Tensor], ...]]


def _move(t: Optional[Tensor], device: torch.device) -> Optional[Tensor]:
    if t is None:
        return None
    out = t.detach().to(device)
    if t.requires_grad:
        out.requires_grad_()
    return out


def to(device: torch.device, value: Optional[TensorOrTensors]) -> Optional[TensorOrTensors]:
    if value is None:
        return None
    if isinstance(value, tuple):
        return tuple(_move(v, device) for v in value)
    return _move(value, device)
