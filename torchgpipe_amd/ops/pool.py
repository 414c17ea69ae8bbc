"""AmoebaNet's 3×3 average pools on a HIP kernel, with the node sum folded in.

:class:`AvgPool3x3` is ``nn.AvgPool2d(3, stride, padding=1, count_include_pad=False)``
(every pool of the reference genotype, ``benchmarks/models/amoebanet/operations.py:50-59``)
whose fp32 GPU path is ``csrc/pool.hip``; ``forward(x, add)`` returns
``pool(x) + add`` from the same pass (``left + right`` of a cell node).
"""
from typing import Optional, Tuple

import torch
from torch import Tensor, nn
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext

__all__ = ['AvgPool3x3']


class _AvgPool3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, add: Optional[Tensor], stride: int) -> Tensor:  # type: ignore[override]
        ctx.shape = (x.shape[2], x.shape[3])
        ctx.stride = stride
        ctx.has_add = add is not None
        return _ext.require(x).avgpool3_forward(x, stride, add)

    @staticmethod
    def backward(ctx, dy: Tensor) -> Tuple:  # type: ignore[override]
        h, w = ctx.shape
        dx = _ext.require(dy).avgpool3_backward(dy, h, w, ctx.stride)
        return dx, (dy if ctx.has_add else None), None


class AvgPool3x3(nn.AvgPool2d):
    """3×3 / padding 1 / ``count_include_pad=False`` average pool (stride 1 or 2)."""

    def __init__(self, stride: int = 1) -> None:
        super().__init__(3, stride=stride, padding=1, count_include_pad=False)

    def forward(self, x: Tensor, add: Optional[Tensor] = None) -> Tensor:  # type: ignore[override]
        stride = self.stride if isinstance(self.stride, int) else self.stride[0]
        if (x.is_cuda and x.dtype == torch.float32 and x.dim() == 4 and stride in (1, 2)
                and _ext.available() and (add is None or add.dtype == torch.float32)):
            return _AvgPool3.apply(x, add, stride)
        out = F.avg_pool2d(x, 3, stride, 1, count_include_pad=False)
        return out if add is None else out + add
