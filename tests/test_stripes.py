"""The multi-path transfer planner (``parallel/stripes.py``): pieces and relay choice."""
import pytest

from torchgpipe_amd.parallel.stripes import Send, message_kind, pieces, plan


@pytest.mark.parametrize('nbytes', [0, 1, 255, 256, 1000, 4096, 10 ** 6, 226_492_416])
@pytest.mark.parametrize('relays', [0, 1, 2, 3])
def test_pieces_tile_the_message(nbytes, relays):
    got = pieces(nbytes, relays)
    pos = 0
    for off, n, path in got:
        assert off == pos and n > 0 and 0 <= path <= relays
        assert off % 256 == 0
        pos += n
    assert pos == nbytes
    # each detour's share is cut into at most 4 forwarded pieces
    for k in range(1, relays + 1):
        assert sum(1 for _, _, p in got if p == k) <= 4


def test_pieces_balance_the_paths():
    """The direct link carries (sub+1)/sub of each detour's share: a detour stores and
    forwards, so its time is (sub+1)/sub of its share's one-link time."""
    nbytes = 400 * 2 ** 20
    got = pieces(nbytes, 3, sub=4)
    share = {k: sum(n for _, n, p in got if p == k) for k in range(4)}
    unit = nbytes / (1.25 + 3)
    assert share[0] == pytest.approx(1.25 * unit, rel=1e-4)
    for k in (1, 2, 3):
        assert share[k] == pytest.approx(unit, rel=1e-4)


def test_message_kind():
    assert message_kind(('sig', True, True, 'skip', 0, 1, 6)) == 'skip'
    assert message_kind(('x', 1)) is None


def _chain(n, sizes, skips=()):
    """Sends of an n-stage chain: activation j -> j+1 of sizes[j], skips (src, dst, bytes),
    and the gradients back; two micro-batches."""
    sends = {j: [] for j in range(n)}
    for _ in range(2):
        for j in range(n - 1):
            sends[j].append(Send(j + 1, 'act', sizes[j]))
        for src, dst, b in skips:
            sends[src].append(Send(dst, 'skip', b))
    for _ in range(2):
        for j in range(n - 1):
            sends[j + 1].append(Send(j, 'gact', sizes[j]))
        for src, dst, b in skips:
            sends[dst].append(Send(src, 'gskip', b))
    return sends


def test_plan_relays_only_over_idle_link_directions():
    sends = _chain(8, [300, 200, 10, 10, 10, 10, 10], skips=[(1, 6, 250)])
    stripes, jobs = plan(sends, list(range(8)), min_bytes=100)
    forward = {(j, j + 1) for j in range(7)} | {(1, 6)}
    assert set(stripes) >= {(0, 1), (1, 0), (1, 2), (2, 1), (1, 6), (6, 1)}
    seen = set()
    for (src, dst), relays in stripes.items():
        assert relays == stripes[(dst, src)]  # gradients come back the same way
        for r in relays:
            assert r not in (src, dst)
            if src < dst:
                # no (large) forward message uses a detour's direction (nor, mirrored, a
                # gradient the backward detour's): only the 10-byte ones may
                for link in ((src, r), (r, dst)):
                    assert link not in forward or link not in {(0, 1), (1, 2), (1, 6)}
                for pair in (frozenset((src, r)), frozenset((r, dst))):
                    assert pair not in seen  # a GPU pair carries one route's detour
                    seen.add(pair)
    # small routes stay direct
    assert (3, 4) not in stripes
    # every relay of every route has a job with its pieces of both directions
    for (src, dst), relays in stripes.items():
        if src > dst:
            continue
        for k, r in enumerate(relays, start=1):
            job = [j for j in jobs[r] if (j.src, j.dst) == (src, dst)]
            assert len(job) == 1
            fwd = [m.nbytes for m in sends[src] if m.dst == dst and m.nbytes >= 100]
            want = [n for b in fwd for _, n, p in pieces(b, len(relays)) if p == k]
            assert list(job[0].forward) == want
            assert len(job[0].backward) == len(job[0].forward)


def test_plan_spreads_relays_over_routes():
    """Two routes of similar size both get detours (relays go one at a time to the route
    whose direct link carries the most), not one route all of them."""
    sends = _chain(8, [151, 10, 10, 10, 10, 10, 10], skips=[(1, 7, 150)])
    stripes, _ = plan(sends, list(range(8)), min_bytes=100, max_relays=3)
    assert stripes.get((0, 1)) and stripes.get((1, 7))


def test_plan_is_deterministic_and_respects_thresholds():
    sends = _chain(4, [50, 60, 70])
    assert plan(sends, [0, 1, 2, 3], min_bytes=100) == ({}, {})
    a = plan(sends, [0, 1, 2, 3], min_bytes=1)
    b = plan({k: list(v) for k, v in reversed(list(sends.items()))}, [0, 1, 2, 3], 1)
    assert a == b


def test_plan_skips_routes_with_other_traffic():
    sends = _chain(4, [500, 10, 10])
    sends[0].append(Send(1, 'other', 500))
    stripes, _ = plan(sends, [0, 1, 2, 3], min_bytes=100)
    assert (0, 1) not in stripes


def test_p2p_refuses_a_step_that_sends_differently_from_its_plan():
    """A striped route checks every message against the plan recorded for its signature:
    a different size (or one message too many) raises instead of mis-delivering pieces,
    and a step that sends fewer messages than planned raises at its end."""
    import torch

    from torchgpipe_amd.parallel.p2p import P2P, StripePlan
    p2p = P2P(torch.device('cpu'))
    p2p.me = 0
    plan = StripePlan({(0, 1): [2], (1, 0): [2]}, {(0, 1): [1024, 1024]}, [], min_bytes=1)
    p2p.use_plan(plan)
    assert p2p._striped(0, 1, 1024, 'k0')
    with pytest.raises(RuntimeError, match='expects 1024'):
        p2p._striped(0, 1, 512, 'k1')
    p2p.use_plan(plan)
    assert p2p._striped(0, 1, 1024, 'k0') and p2p._striped(0, 1, 1024, 'k1')
    with pytest.raises(RuntimeError, match='no message'):
        p2p._striped(0, 1, 1024, 'k2')
    # messages under the threshold and unplanned routes go direct
    p2p.use_plan(StripePlan({(0, 1): [2]}, {(0, 1): [4096]}, [], min_bytes=2048))
    assert not p2p._striped(0, 1, 100, 'small')
    assert not p2p._striped(0, 3, 1 << 20, 'other route')
    with pytest.raises(RuntimeError, match='sent 0 messages this step, the stripe plan 1'):
        p2p.end_relays()


def test_plan_uses_the_reverse_direction_of_busy_links():
    """U-Net p4 at the reference balance (routes 0->1, 1->2, 2->3 and skips 0->3, 1->2,
    1->3) has no detour whose links are idle in both directions, so an undirected planner
    finds none; the forward phase leaves 2 -> 1 and 3 -> 1 free (only gradients use them,
    later), so the large first boundary goes 0 -> 2 -> 1 and 0 -> 3 -> 1 too (0 -> 3
    carries a small skip only)."""
    sends = _chain(4, [500, 10, 10], skips=[(0, 3, 10), (1, 2, 10), (1, 3, 10)])
    stripes, jobs = plan(sends, [0, 1, 2, 3], min_bytes=100)
    assert stripes == {(0, 1): [2, 3], (1, 0): [2, 3]}
    assert [(j.src, j.dst) for j in jobs[2]] == [(0, 1)]


def test_plan_shares_a_lightly_loaded_link_direction():
    """U-Net p4's 302 MB skip 0 -> 3: every link into stage 3 carries forward traffic, so no
    idle detour exists; 2 -> 3 carries only the 38 MB activation (1/8 of the skip), so the
    skip still takes 0 -> 2 -> 3.  A busier link (half the message) is not shared."""
    sends = _chain(4, [151, 75, 37], skips=[(0, 3, 302), (1, 2, 10), (1, 3, 151)])
    stripes, _ = plan(sends, [0, 1, 2, 3], min_bytes=100)
    assert 2 in stripes[(0, 3)]
    sends = _chain(4, [151, 75, 151], skips=[(0, 3, 302), (1, 2, 10), (1, 3, 151)])
    stripes, _ = plan(sends, [0, 1, 2, 3], min_bytes=100)
    assert (0, 3) not in stripes
