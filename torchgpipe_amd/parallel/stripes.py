"""Multi-path ("striped") transfers: large messages split over relays through idle GPUs.

An 8-GPU MI355X node is a fully connected xGMI mesh: every pair of GPUs has its own link,
and RCCL point-to-point between two GPUs moves data over that one link.  A pipeline uses
only a few of the 28 links -- the chain of neighbouring stages and the skip routes -- and
its first boundaries carry more bytes per micro-batch than one link moves in a forward
cell (U-Net(5,64) p8: 226 MB of skips from stage 1 to stage 6 per micro-batch, AmoebaNet
n8m32: 321 MB from stage 0 to 1; ``profiles/r5/speedup_prediction.md``).  Striping sends
chunk 0 of such a message over the direct link and chunk k over ``src -> relay_k ->
dst``, where both link directions of the detour carry no forward pipeline traffic, so a
route gets up to ``1 + max_relays`` links' bandwidth.  xGMI links are full duplex, and a
GPipe step's forward transfers (upward in rank order) and gradient transfers (downward)
happen in two phases that never overlap: a detour may run against the direction of a busy
pipeline link (U-Net p4 has no fully idle detour; ``tests/test_stripes.py``).

Plan.  Every rank records the messages it sends in one training step (destination, kind,
bytes, in order); at the start of the next step of the same signature the ranks exchange
those lists on the control group and compute the same plan: forward routes (src, dst)
(activations and skips; gradients only the other way) with a message of at least
``min_bytes``, largest first, each taking relays whose two link directions carry no
forward message and whose GPU pairs no other route's detour uses yet; the route's
gradients (``dst -> src``) take the same relays back, over the mirrored directions, which
the backward phase leaves free for the same reason.
Every message of at least ``min_bytes`` on a striped route travels in pieces (both ends
know its size from the shape metadata); smaller ones stay on the direct link.  A relay
link therefore carries one route, forward pieces then gradient pieces, exactly in the
order the endpoints post them.

Relay.  A relay posts, per step and route, ``recv(chunk from src) -> send(chunk to dst)``
for every forward message, then the same for the gradients in backward order, on a
process group of its own (``relay_group``) and, with RCCL, on a stream of its own per
route: the chain is stream-ordered (a receive's completion gates the send; a staging
slot is reused only after its previous send completed), so the relay's host posts the
whole step up front and its compute streams never wait on relay traffic.  With gloo a
thread per route runs the same chain with blocking waits.
"""
from typing import Dict, Hashable, List, NamedTuple, Optional, Sequence, Tuple

__all__ = ['Send', 'RelayJob', 'pieces', 'message_kind', 'plan']

STRIPED_KINDS = ('act', 'skip')
# a detour may share a link direction with forward traffic of at most this fraction of
# the striped message (see plan)
SHARE_RATIO = 8
GRAD_KINDS = ('gact', 'gskip')


class Send(NamedTuple):
    """One message a rank sent in a step (recorded in send order)."""
    dst: int
    kind: str
    nbytes: int


class RelayJob(NamedTuple):
    """What a relay forwards for one route per step: the sizes of its pieces of the
    ``src -> dst`` messages in their order, then of the ``dst -> src`` gradients."""
    src: int
    dst: int
    forward: Tuple[int, ...]
    backward: Tuple[int, ...]


def message_kind(key: Hashable) -> Optional[str]:
    """The kind (``act``, ``skip``, ``gact``, ``gskip``...) of a pipeline message key
    ``(signature, training, grad, kind, i, src, dst)``; ``None`` for other keys."""
    if isinstance(key, tuple) and len(key) == 7 and isinstance(key[3], str):
        return key[3]
    return None


def pieces(nbytes: int, n_relays: int, sub: int = 4,
           align: int = 256) -> List[Tuple[int, int, int]]:
    """How a ``nbytes`` message travels over the direct link and ``n_relays`` detours:
    ``(offset, size, path)`` pieces, path 0 = direct, path k = through relay k.

    A relay stores and forwards, so each detour's share is cut into ``sub`` pieces that
    it forwards as they arrive (its time is ``(sub + 1) / sub`` of its share's one-link
    time); the direct link carries that much more than each detour so that every path
    finishes together.  Cuts are ``align``-byte aligned; empty pieces are dropped.
    """
    if n_relays <= 0:
        return [(0, nbytes, 0)] if nbytes else []

    def up(x: float) -> int:
        return min(nbytes, -(-int(x) // align) * align)

    w0 = (sub + 1) / sub
    unit = nbytes / (w0 + n_relays)
    cuts = [0, up(unit * w0)] + [up(unit * (w0 + k)) for k in range(1, n_relays)] + [nbytes]
    out: List[Tuple[int, int, int]] = []
    if cuts[1] > 0:
        out.append((0, cuts[1], 0))
    for k in range(1, n_relays + 1):
        lo, hi = cuts[k], cuts[k + 1]
        step = -(-(hi - lo) // sub)
        step = -(-step // align) * align
        pos = lo
        while pos < hi:
            n = min(step, hi - pos)
            out.append((pos, n, k))
            pos += n
    return out


def plan(sends: Dict[int, Sequence[Send]], ranks: Sequence[int], min_bytes: int,
         max_relays: int = 3, sub: int = 4) -> Tuple[Dict[Tuple[int, int], List[int]],
                                       Dict[int, List[RelayJob]]]:
    """Stripes ``{(src, dst): [relays]}`` (gradient directions included) and each relay's
    jobs, from every rank's recorded sends of one step.  Deterministic: every rank that
    calls it with the same lists gets the same plan."""
    routes: Dict[Tuple[int, int], List[Send]] = {}
    for src in sorted(sends):
        for s in sends[src]:
            routes.setdefault((src, s.dst), []).append(s)
    # Forward-phase directed links: every forward message travels upward-ordered routes
    # (activations j -> j+1, skips stash -> pop) and its gradient the reverse direction in
    # the backward phase, which starts only after the last stage's last forward -- so the
    # two phases never overlap in time, and a detour link direction is free when no forward
    # route uses it (the mirrored gradient detour is then free in the backward phase).
    # A GPU pair carries at most one route's detour: its relay communicator orders that
    # route's forward then backward pieces, and a second route on it would queue behind.
    # A direction that carries a small forward route (at most 1/SHARE_RATIO of the striped
    # message: U-Net p4's 38 MB activation 2 -> 3 beside its 302 MB skip 0 -> 3, whose
    # destination has no other way in) still takes a detour: the link has the room.
    fwd_load = {r: max(m.nbytes for m in msgs) for r, msgs in routes.items()
                if not {m.kind for m in msgs} <= set(GRAD_KINDS)}
    candidates = []
    for (src, dst), msgs in routes.items():
        if not {m.kind for m in msgs} <= set(STRIPED_KINDS):
            continue
        back = routes.get((dst, src), [])
        if not {m.kind for m in back} <= set(GRAD_KINDS):
            continue  # the reverse direction carries something else too
        size = max(m.nbytes for m in msgs)
        if size < min_bytes:
            continue
        candidates.append((-size, src, dst))
    relay_pairs: set = set()
    # relays one at a time, each to the route whose direct link then still carries the
    # most bytes (size * w0 / (w0 + R)): a large route does not take every free detour
    # while another one of nearly its size gets none
    w0 = (sub + 1) / sub
    chosen: Dict[Tuple[int, int], List[int]] = {(src, dst): [] for _, src, dst in candidates}
    size_of = {(src, dst): -neg for neg, src, dst in candidates}
    open_routes = set(chosen)
    while open_routes:
        src, dst = max(open_routes, key=lambda r: (size_of[r] * w0 / (w0 + len(chosen[r])),
                                                   -r[0], -r[1]))
        relays = chosen[(src, dst)]
        # relays nearest the route's midpoint first (any order works; this one is fixed)
        order = sorted((r for r in ranks if r not in (src, dst)),
                       key=lambda r: (abs(2 * r - src - dst), r))
        room = size_of[(src, dst)] / SHARE_RATIO
        pick = next((r for r in order if fwd_load.get((src, r), 0) <= room
                     and fwd_load.get((r, dst), 0) <= room
                     and frozenset((src, r)) not in relay_pairs
                     and frozenset((r, dst)) not in relay_pairs), None)
        if pick is None:
            open_routes.discard((src, dst))
            continue
        relay_pairs.add(frozenset((src, pick)))
        relay_pairs.add(frozenset((pick, dst)))
        relays.append(pick)
        if len(relays) >= max_relays:
            open_routes.discard((src, dst))
    stripes: Dict[Tuple[int, int], List[int]] = {}
    jobs: Dict[int, List[RelayJob]] = {}
    for _, src, dst in sorted(candidates):
        relays = chosen[(src, dst)]
        if not relays:
            continue
        stripes[(src, dst)] = relays
        back = [m.nbytes for m in routes.get((dst, src), []) if m.nbytes >= min_bytes]
        if back:
            stripes[(dst, src)] = relays
        fwd = [m.nbytes for m in routes[(src, dst)] if m.nbytes >= min_bytes]

        def mine(sizes: List[int], k: int) -> Tuple[int, ...]:
            return tuple(n for size in sizes
                         for _, n, path in pieces(size, len(relays), sub) if path == k)

        for k, r in enumerate(relays, start=1):
            jobs.setdefault(r, []).append(RelayJob(src, dst, mine(fwd, k), mine(back, k)))
    return stripes, jobs
