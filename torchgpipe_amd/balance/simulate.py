"""Discrete-event model of a GPipe fill-drain step, for choosing balances.

Given per-layer forward / backward device times (``benchmarks/layer_profile.py``),
a balance and the micro-batch count, :func:`step_time` returns the simulated
time of one multi-process training step:

* forward cell ``(i, j)`` starts when stage ``j`` is free, the activation of
  ``(i, j-1)`` has crossed the ``j-1 → j`` link, and every skip tensor popped
  in stage ``j`` has crossed its own (direct) link;
* backward cells run in reverse micro-batch order; a checkpointed cell
  recomputes as soon as its stage is free (before its gradient arrives), then
  waits for the output gradient and the gradients of the skips it stashed;
* every directed link is a FIFO resource moving ``bytes / link_GBps``.

:func:`optimize` searches balances that minimise the simulated step time,
starting from the min-max partition of per-cell cost, with boundary moves.
"""
from typing import Dict, List, Optional, Sequence, Tuple

from torchgpipe_amd.balance import blockpartition

__all__ = ['step_time', 'optimize']

Skip = Tuple[int, int, float]  # (stash layer, pop layer, bytes)


def _owner(balance: Sequence[int]) -> List[int]:
    owner: List[int] = []
    for j, b in enumerate(balance):
        owner += [j] * b
    return owner


def step_time(fwd: Sequence[float], bwd: Sequence[float], balance: Sequence[int], m: int,
              checkpoint: str = 'except_last', out_bytes: Optional[Sequence[float]] = None,
              skips: Sequence[Skip] = (), link_gbps: Optional[float] = None) -> float:
    """Simulated milliseconds of one step (forward + backward of ``m`` micro-batches)."""
    n = len(balance)
    owner = _owner(balance)
    F = [0.0] * n
    B = [0.0] * n
    for layer, j in enumerate(owner):
        F[j] += fwd[layer]
        B[j] += bwd[layer]
    stop = {'always': m, 'except_last': m - 1, 'never': 0}[checkpoint]

    def xfer(nbytes: float) -> float:
        return 0.0 if not link_gbps else nbytes / (link_gbps * 1e6)

    # Boundary activation sizes and cross-stage skip routes.
    act = [0.0] * n
    if out_bytes is not None:
        end = 0
        for j, b in enumerate(balance):
            end += b
            act[j] = float(out_bytes[end - 1])
    routes = [(owner[s], owner[p], nbytes) for s, p, nbytes in skips if owner[s] != owner[p]]

    link_free: Dict[Tuple[int, int], float] = {}

    def send(src: int, dst: int, t: float, nbytes: float) -> float:
        start = max(t, link_free.get((src, dst), 0.0))
        done = start + xfer(nbytes)
        link_free[(src, dst)] = done
        return done

    free = [0.0] * n
    f_done = [[0.0] * n for _ in range(m)]
    arrive: Dict[Tuple[int, int], float] = {}  # (i, j) -> all inputs of cell arrived
    for i in range(m):
        for j in range(n):
            ready = arrive.get((i, j), 0.0)
            start = max(ready, free[j])
            f_done[i][j] = free[j] = start + F[j]
            if j + 1 < n:
                t = send(j, j + 1, f_done[i][j], act[j])
                arrive[(i, j + 1)] = max(arrive.get((i, j + 1), 0.0), t)
            for src, dst, nbytes in routes:
                if src == j:
                    t = send(src, dst, f_done[i][j], nbytes)
                    arrive[(i, dst)] = max(arrive.get((i, dst), 0.0), t)

    garrive: Dict[Tuple[int, int], float] = {}
    for i in reversed(range(m)):
        for j in reversed(range(n)):
            rc_done = free[j] + (F[j] if i < stop else 0.0)
            start = max(rc_done, garrive.get((i, j), 0.0))
            free[j] = start + B[j]
            if j > 0:
                t = send(j, j - 1, free[j], act[j - 1])
                garrive[(i, j - 1)] = max(garrive.get((i, j - 1), 0.0), t)
            for src, dst, nbytes in routes:
                if dst == j:
                    t = send(dst, src, free[j], nbytes)
                    garrive[(i, src)] = max(garrive.get((i, src), 0.0), t)
    return max(free)


def optimize(fwd: Sequence[float], bwd: Sequence[float], n: int, m: int,
             checkpoint: str = 'except_last', out_bytes: Optional[Sequence[float]] = None,
             skips: Sequence[Skip] = (), link_gbps: Optional[float] = None,
             start: Optional[Sequence[int]] = None, rounds: int = 500
             ) -> Tuple[List[int], float]:
    """Local search over balances (boundary moves of 1..4 layers)."""
    def cost(bal: Sequence[int]) -> float:
        return step_time(fwd, bwd, bal, m, checkpoint, out_bytes, skips, link_gbps)

    cell = [2 * f + b for f, b in zip(fwd, bwd)]
    candidates = [blockpartition.solve_splits([c * 1000 for c in cell], n)]
    if start is not None:
        candidates.append(list(start))
    best, best_t = None, float('inf')
    for cand in candidates:
        t = cost(cand)
        if t < best_t:
            best, best_t = list(cand), t
    assert best is not None
    for _ in range(rounds):
        improved = False
        for k in range(n - 1):
            for delta in (-4, -2, -1, 1, 2, 4):
                cand = list(best)
                cand[k] += delta
                cand[k + 1] -= delta
                if min(cand) < 1:
                    continue
                t = cost(cand)
                if t < best_t - 1e-9:
                    best, best_t, improved = cand, t, True
        if not improved:
            break
    return best, best_t
