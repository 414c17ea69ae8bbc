"""U-Net resolution changes on HIP kernels (``csrc/unet_ops.hip``).

* :func:`up2x_cat` -- ``cat(nearest_upsample_2x(x), skip)``: the decoder's ``up`` +
  ``skip`` layers (reference ``benchmarks/models/unet/__init__.py``: ``nn.Upsample`` then
  ``torch.cat`` in the skip pop) as one pass; the backward reads the upsampled part of the
  concatenation's gradient in place and hands ``skip`` its channel slice (a view).
* :class:`MaxPool2x2` -- ``nn.MaxPool2d(2, stride=2)`` without ATen's int64 index tensor;
  the backward re-finds each window's argmax from the input (ATen's tie / NaN order).

Both fall back to the PyTorch ops off the GPU, for other dtypes and odd shapes.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor, nn
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext

__all__ = ['up2x_cat', 'MaxPool2x2']


class _Up2xCat(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, skip: Tensor) -> Tensor:  # type: ignore[override]
        ctx.c1 = x.shape[1]
        return _ext.require(x).up2x_cat_forward(x, skip)

    @staticmethod
    def backward(ctx, dy: Tensor) -> Tuple[Tensor, Tensor]:  # type: ignore[override]
        dx = _ext.require(dy).up2x_backward(dy, ctx.c1)
        return dx, dy[:, ctx.c1:]


def _fusable(*ts: Tensor) -> bool:
    return all(t.is_cuda and t.dtype == torch.float32 and t.dim() == 4 for t in ts) \
        and _ext.available()


def up2x_cat(x: Tensor, skip: Tensor) -> Tensor:
    """``torch.cat((upsample_nearest_2x(x), skip), 1)``, zero-padding the upsampled part
    to ``skip``'s size if they differ (odd sizes), like the reference's skip pop."""
    if _fusable(x, skip) and skip.shape[0] == x.shape[0] and \
            tuple(skip.shape[2:]) == (2 * x.shape[2], 2 * x.shape[3]):
        return _Up2xCat.apply(x, skip)
    up = F.interpolate(x, scale_factor=2, mode='nearest')
    if up.shape[2:] != skip.shape[2:]:
        pad = []
        for have, want in reversed(list(zip(up.shape[2:], skip.shape[2:]))):
            pad += [0, want - have]
        up = F.pad(up, pad)
    return torch.cat((up, skip), dim=1)


class _MaxPool2x2(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, add: Optional[Tensor]) -> Tensor:  # type: ignore[override]
        ctx.save_for_backward(x)
        ctx.has_add = add is not None
        return _ext.require(x).maxpool2x2_forward(x, add)

    @staticmethod
    def backward(ctx, dy: Tensor):  # type: ignore[override]
        (x,) = ctx.saved_tensors
        return _ext.require(dy).maxpool2x2_backward(x, dy), dy if ctx.has_add else None


class MaxPool2x2(nn.MaxPool2d):
    """``nn.MaxPool2d(2, stride=2)`` (floor mode, no padding / dilation / indices).

    ``forward(x, add)`` returns ``pool(x) + add`` in the same pass (AmoebaNet's cell-node
    sums, ``models/amoebanet.py``); the backward reads a channel-sliced gradient in place.
    """

    def __init__(self) -> None:
        super().__init__(2, stride=2)

    def forward(self, x: Tensor, add: Optional[Tensor] = None) -> Tensor:  # type: ignore[override]
        if _fusable(x) and not self.return_indices and not self.ceil_mode and \
                (add is None or _fusable(add)):
            return _MaxPool2x2.apply(x, add)
        out = super().forward(x)
        return out if add is None else out + add
