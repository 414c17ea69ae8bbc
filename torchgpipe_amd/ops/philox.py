"""Bit-exact PyTorch (CPU) reference of the HIP Philox4x32-10 stream.

Mirrors ``csrc/philox.h``: key = (seed_lo, seed_hi ^ 0x7467706D), counter =
(index_lo, index_hi, offset_lo, offset_hi), uniform = (word >> 8) * 2^-24.
Used as the oracle in kernel tests and as the CPU implementation of the
framework dropout ops.
"""
from typing import List

import torch
from torch import Tensor

__all__ = ['philox4x32_10', 'uniform']

_M0 = 0xD2511F53
_M1 = 0xCD9E8D57
_W0 = 0x9E3779B9
_W1 = 0xBB67AE85
_DOMAIN = 0x7467706D
_MASK = 0xFFFFFFFF


def philox4x32_10(index: Tensor, offset: int, seed: int) -> List[Tensor]:
    """Return the four 32-bit words (as int64 tensors) for each counter index."""
    index = index.to(torch.int64)
    c0 = index & _MASK
    c1 = (index >> 32) & _MASK
    offset &= 0xFFFFFFFFFFFFFFFF
    seed &= 0xFFFFFFFFFFFFFFFF
    c2 = torch.full_like(c0, offset & _MASK)
    c3 = torch.full_like(c0, (offset >> 32) & _MASK)
    k0 = seed & _MASK
    k1 = ((seed >> 32) & _MASK) ^ _DOMAIN
    for _ in range(10):
        # 32x32-bit products can exceed int64: split them into 16-bit halves.
        lo0, hi0 = _mul32(c0, _M0)
        lo1, hi1 = _mul32(c2, _M1)
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
        k0 = (k0 + _W0) & _MASK
        k1 = (k1 + _W1) & _MASK
    return [c0, c1, c2, c3]


def _mul32(a: Tensor, m: int):  # type: ignore[no-untyped-def]
    """32x32→64-bit product of uint32 values held in int64, as (lo, hi) words."""
    a_lo = a & 0xFFFF
    a_hi = a >> 16
    m_lo = m & 0xFFFF
    m_hi = m >> 16
    ll = a_lo * m_lo
    lh = a_lo * m_hi
    hl = a_hi * m_lo
    hh = a_hi * m_hi
    mid = (ll >> 16) + (lh & 0xFFFF) + (hl & 0xFFFF)
    lo = ((mid & 0xFFFF) << 16) | (ll & 0xFFFF)
    hi = hh + (lh >> 16) + (hl >> 16) + (mid >> 16)
    return lo & _MASK, hi & _MASK


def to_uniform(word: Tensor) -> Tensor:
    return (word >> 8).to(torch.float32) * (1.0 / 16777216.0)


def uniform(n: int, seed: int, offset: int) -> Tensor:
    """``n`` uniforms in [0, 1) exactly as ``philox_uniform_kernel`` produces them."""
    quads = (n + 3) // 4
    words = philox4x32_10(torch.arange(quads, dtype=torch.int64), offset, seed)
    out = torch.stack([to_uniform(w) for w in words], dim=1).reshape(-1)
    return out[:n]
