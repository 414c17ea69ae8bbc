"""Small device utilities: spin kernel (K5) and multi-tensor pack/unpack (K6)."""
from typing import List, Sequence

import torch
from torch import Tensor

from torchgpipe_amd.ops import _ext

__all__ = ['spin', 'pack', 'unpack', 'philox_uniform']


def spin(seconds: float, device: torch.device) -> None:
    """Enqueue a kernel that busy-waits ``seconds`` of wall time on ``device``'s stream.

    The HIP counterpart of ``torch.cuda._sleep`` used by race-provoking tests
    (reference ``tests/conftest.py:10-26``); it is calibrated in nanoseconds
    (``s_memrealtime`` runs at a constant 100 MHz), so no cycles-per-ms probe
    is needed.
    """
    _ext.require().spin(int(seconds * 1e9), device)


def philox_uniform(n: int, seed: int, offset: int, device: torch.device) -> Tensor:
    return _ext.require().philox_uniform(n, seed, offset, device)


def pack(tensors: Sequence[Tensor], out: Tensor) -> Tensor:
    """Copy ``tensors`` back to back into the flat byte buffer ``out`` (one launch)."""
    views: List[Tensor] = []
    pos = 0
    for t in tensors:
        nbytes = t.numel() * t.element_size()
        views.append(out[pos:pos + nbytes])
        pos = (pos + nbytes + 15) // 16 * 16  # keep every segment 16-byte aligned
    srcs = [t.contiguous().view(-1).view(torch.uint8) for t in tensors]
    if out.is_cuda:
        _ext.require(out).copy_segments(srcs, views)
    else:
        for s, v in zip(srcs, views):
            v.copy_(s)
    return out


def packed_nbytes(tensors: Sequence[Tensor]) -> int:
    pos = 0
    for t in tensors:
        pos = (pos + t.numel() * t.element_size() + 15) // 16 * 16
    return pos


def unpack(buf: Tensor, outs: Sequence[Tensor]) -> None:
    """Inverse of :func:`pack`: scatter the flat buffer into the (contiguous) ``outs``."""
    srcs: List[Tensor] = []
    dsts: List[Tensor] = []
    pos = 0
    for t in outs:
        nbytes = t.numel() * t.element_size()
        srcs.append(buf[pos:pos + nbytes])
        dsts.append(t.view(-1).view(torch.uint8))
        pos = (pos + nbytes + 15) // 16 * 16
    if buf.is_cuda:
        _ext.require(buf).copy_segments(srcs, dsts)
    else:
        for s, d in zip(srcs, dsts):
            d.copy_(s)
