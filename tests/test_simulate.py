"""balance/simulate.py: the GPipe step model used for transfer-inclusive predictions,
against fill/drain schedules worked out by hand."""
import pytest

from torchgpipe_amd.balance.simulate import optimize, step_time


def test_no_transfer_never_is_m_plus_n_minus_one_cells():
    # 2 stages, 2 micro-batches, F = 1, B = 2, no recomputation: forward 0-3, stage 1's
    # backwards 3-5 / 5-7, stage 0's 5-7 / 7-9
    assert step_time([1, 1], [2, 2], [1, 1], 2, 'never') == pytest.approx(9.0)
    # (m + n - 1) (F + B) in general, for equal stages
    assert step_time([1] * 4, [2] * 4, [1] * 4, 8, 'never') == pytest.approx(11 * 3)


def test_recompute_runs_before_the_gradient_arrives():
    # 'always': stage 0 recomputes micro-batch 1 at 2-3 while stage 1 works (the reference's
    # Recompute-before-Wait), so only micro-batch 0's recompute (8-9) is exposed: 11
    assert step_time([1, 1], [2, 2], [1, 1], 2, 'always') == pytest.approx(11.0)
    # except_last: the last micro-batch keeps its activations
    assert step_time([1, 1], [2, 2], [1, 1], 2, 'except_last') == pytest.approx(10.0)


def test_link_transfers_delay_the_consumer():
    # 1e6 bytes at 1 GB/s = 1 ms per hop, in each direction:
    # forward (0,0) 0-1, hop 1-2, (0,1) 2-3; (1,0) 1-2, hop 2-3, (1,1) 3-4;
    # backward (1,1) 4-6, hop 6-7, (1,0) 7-9; (0,1) 6-8, hop 8-9, (0,0) 9-11
    t = step_time([1, 1], [2, 2], [1, 1], 2, 'never', out_bytes=[1e6, 0.0], link_gbps=1.0)
    assert t == pytest.approx(11.0)
    assert step_time([1, 1], [2, 2], [1, 1], 2, 'never', out_bytes=[1e6, 0.0]) == \
        pytest.approx(9.0)  # no bandwidth given: free transfers


def test_skip_routes_use_their_own_link():
    # 3 stages of F = 1, B = 1, one micro-batch; a 2 ms skip 0 -> 2 on its own link
    base = step_time([1, 1, 1], [1, 1, 1], [1, 1, 1], 1, 'never')
    assert base == pytest.approx(6.0)
    skip = step_time([1, 1, 1], [1, 1, 1], [1, 1, 1], 1, 'never', skips=[(0, 2, 2e6)],
                     link_gbps=1.0)
    # the skip leaves stage 0 at 1 and lands at 3 (stage 2 would start at 2): stage 2 runs
    # 3-4 forward, 4-5 backward; its gradient lands on stage 0 at 7 (stage 1's at 6):
    # stage 0's backward 7-8
    assert skip == pytest.approx(8.0)


def test_optimize_finds_the_balanced_split():
    fwd = [1.0, 1.0, 1.0, 3.0, 1.0, 1.0]
    bwd = [2 * f for f in fwd]
    bal, t = optimize(fwd, bwd, 2, 8, 'never')
    assert sum(bal) == 6 and bal == [3, 3]
    assert t == pytest.approx(step_time(fwd, bwd, bal, 8, 'never'))
