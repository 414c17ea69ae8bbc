"""Contiguous block partitioning of a cost sequence (min-max, then least variance).

The reference uses the Bárány et al. *block partitions of sequences*
heuristic (``torchgpipe/balance/blockpartition.py:11-89``), which normalises
costs to [0, 1] and stops as soon as ``max ≤ min + 1`` — a loose criterion.
Here the partition is **exact**: a dynamic program finds the smallest
achievable maximum block cost, then a second DP picks, among all partitions
with that maximum, the one with the least sum of squared block costs (i.e.
the most even one).  Both DPs are vectorised with numpy: O(k·n²) work,
milliseconds even for 2 000-layer models on 8 partitions.
"""
from typing import List, Sequence

import numpy as np

__all__ = ['solve', 'solve_splits']


def _validate(sequence: Sequence[float], partitions: int) -> None:
    if partitions < 1:
        raise ValueError(f'partitions must be a positive integer ({partitions} < 1)')
    if len(sequence) < partitions:
        raise ValueError('sequence is shorter than intended partitions '
                         f'({len(sequence)} < {partitions})')


def solve_splits(sequence: Sequence[float], partitions: int = 1) -> List[int]:
    """Return the block sizes (lengths) of the optimal partition."""
    _validate(sequence, partitions)
    n = len(sequence)
    k = partitions
    cost = np.asarray(sequence, dtype=np.float64)
    prefix = np.concatenate([[0.0], np.cumsum(cost)])
    inf = np.inf

    # seg[t, i] = cost of block (t, i]  for t < i
    seg = prefix[None, :] - prefix[:, None]
    valid = np.triu(np.ones((n + 1, n + 1), dtype=bool), k=1)
    seg = np.where(valid, seg, inf)

    # Pass 1: minimal max block cost.  best[j][i] = optimal max over first i items in j blocks.
    best = np.full(n + 1, inf)
    best[0] = 0.0
    for _ in range(k):
        cand = np.maximum(best[:, None], seg)  # (t, i)
        best = cand.min(axis=0)
        best[0] = inf
    limit = best[n]
    tol = 1e-9 * max(1.0, abs(limit))

    # Pass 2: least sum of squares among partitions whose blocks are all <= limit.
    allowed = np.where(seg <= limit + tol, seg * seg, inf)
    sq = np.full(n + 1, inf)
    sq[0] = 0.0
    choice = np.zeros((k, n + 1), dtype=np.int64)
    for j in range(k):
        cand = sq[:, None] + allowed
        choice[j] = cand.argmin(axis=0)
        sq = cand.min(axis=0)
        sq[0] = inf

    sizes: List[int] = []
    i = n
    for j in range(k - 1, -1, -1):
        t = int(choice[j][i])
        sizes.append(i - t)
        i = t
    sizes.reverse()
    assert i == 0 and all(s > 0 for s in sizes), sizes
    return sizes


def solve(sequence: List[int], partitions: int = 1) -> List[List[int]]:
    """Split ``sequence`` into ``partitions`` contiguous non-empty blocks."""
    sizes = solve_splits(sequence, partitions)
    out: List[List[int]] = []
    start = 0
    for size in sizes:
        out.append(list(sequence[start:start + size]))
        start += size
    return out
