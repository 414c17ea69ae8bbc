"""Fused Dropout2d → InstanceNorm2d → LeakyReLU (the U-Net cell epilogue).

The U-Net benchmark model (``benchmarks/models/unet/__init__.py:42-48`` in the
reference) applies ``Conv2d → Dropout2d(0.1) → InstanceNorm2d → LeakyReLU``
55 times per forward pass.  Unfused, the three epilogue ops cost 4 HBM reads
+ 3 writes forward and 6 reads + 3 writes backward per activation, and keep
two extra full-size activations alive for backward.  The HIP kernel K3
(``csrc/kernels.hip``) holds each (n, c) plane in registers: 1 read + 1 write
forward, 2 reads + 1 write backward, and only the conv output plus three
per-plane scalars are saved.

The Dropout2d channel mask comes from Philox4x32-10 with an explicit
``(seed, offset)`` (``utils.rng.philox_pair``): replayed bit-exactly under
checkpoint recomputation through the cell's RNG tape.

CPU tensors (and non-fp32 dtypes) use a PyTorch composite with the same
Philox mask — the oracle of the kernel tests.
"""
from typing import Optional, Tuple

import torch
from torch import Tensor, nn
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext
from torchgpipe_amd.ops.philox import philox4x32_10, to_uniform
from torchgpipe_amd.utils.rng import philox_draw

__all__ = ['drop_norm_act', 'DropNormAct', 'plane_scale_reference']


def _signed64(v: int) -> int:
    v &= 0xFFFFFFFFFFFFFFFF
    return v - (1 << 64) if v >= (1 << 63) else v


def plane_scale_reference(planes: int, p: float, seed: int, offset: int,
                          device: torch.device) -> Tensor:
    """Per-plane dropout scale (0 or 1/(1-p)) exactly as kernel K3 draws it."""
    word = philox4x32_10(torch.arange(planes, dtype=torch.int64), offset, seed)[0]
    keep = to_uniform(word) >= p
    return (keep.to(torch.float32) / (1.0 - p)).to(device)


def _composite(x: Tensor, p: float, eps: float, slope: float, seed: int, offset: int,
               dropout: bool) -> Tensor:
    n, c = x.shape[:2]
    if dropout:
        scale = plane_scale_reference(n * c, p, seed, offset, x.device).to(x.dtype)
        x = x * scale.view(n, c, *([1] * (x.dim() - 2)))
    y = F.instance_norm(x, eps=eps)
    return F.leaky_relu(y, slope)


class _DropNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x: Tensor, p: float, eps: float, slope: float,  # type: ignore[override]
                seed: int, offset: int, dropout: bool, rng: Optional[Tensor] = None) -> Tensor:
        ops = _ext.require(x)
        y, mean, rstd, scale = ops.dna_forward(x, p, eps, slope, seed, offset, dropout, rng)
        ctx.save_for_backward(x, mean, rstd, scale)
        ctx.slope = slope
        return y

    @staticmethod
    def backward(ctx, dy: Tensor) -> Tuple:  # type: ignore[override]
        x, mean, rstd, scale = ctx.saved_tensors
        dx = _ext.require(dy).dna_backward(dy, x, mean, rstd, scale, ctx.slope)
        return dx, None, None, None, None, None, None, None


def drop_norm_act(x: Tensor, p: float = 0.1, training: bool = True, eps: float = 1e-5,
                  slope: float = 1e-2) -> Tensor:
    """``leaky_relu(instance_norm(dropout2d(x, p)), slope)`` in one HIP kernel."""
    dropout = training and p > 0.0
    n, c = x.shape[:2]
    seed, offset, rng = philox_draw(x.device, n * c) if dropout else (0, 0, None)
    if x.is_cuda and x.dtype == torch.float32:
        return _DropNormAct.apply(x.contiguous(), float(p), float(eps), float(slope),
                                  _signed64(seed), _signed64(offset), dropout, rng)
    if rng is not None:
        raise RuntimeError('drop_norm_act: a device Philox slot needs the fp32 GPU kernel')
    return _composite(x, p, eps, slope, seed, offset, dropout)


class DropNormAct(nn.Module):
    """Module form of :func:`drop_norm_act` (no parameters, no buffers)."""

    def __init__(self, p: float = 0.1, eps: float = 1e-5, negative_slope: float = 1e-2) -> None:
        super().__init__()
        self.p = p
        self.eps = eps
        self.negative_slope = negative_slope

    def extra_repr(self) -> str:
        return f'p={self.p}, eps={self.eps}, negative_slope={self.negative_slope}'

    def forward(self, x: Tensor) -> Tensor:  # type: ignore[override]
        return drop_norm_act(x, self.p, self.training, self.eps, self.negative_slope)
