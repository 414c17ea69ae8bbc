"""The bench.py driver contract: JSON records from rank 0, MAX-over-ranks timing.

Rank 0 prints the complete record right after the headline and re-prints it, augmented,
after every section; every line is a complete record and the last one the most complete.

Runs the script end to end on CPU (gloo) with the ``--tiny`` model variant, at
one rank and under ``torch.distributed.run`` with two ranks.
"""
import json
import os
import socket
import subprocess
import sys
from typing import Optional

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {'metric', 'value', 'unit', 'n_gpus', 'steps', 'warmup', 'ms_per_step',
        'higher_is_better', 'scaling', 'vs_baseline', 'dtype', 'data', 'config'}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _run(nproc: int, *extra: str) -> dict:
    return _run_lines(nproc, *extra)[-1]


def _run_lines(nproc: int, *extra: str, env_extra: Optional[dict] = None) -> list:
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', OMP_NUM_THREADS='2',
               **(env_extra or {}))
    args = ['bench.py', '--gpus', str(nproc), '--steps', '1', '--warmup', '1', '--tiny',
            '--batch', '4', '--chunks', '2', *extra]
    if nproc > 1:
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
               f'--nproc-per-node={nproc}', '--master-addr', '127.0.0.1',
               '--master-port', str(_free_port()), *args]
    else:
        cmd = [sys.executable, *args]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert lines, out.stderr[-3000:]
    records = [json.loads(ln) for ln in lines]  # nothing but JSON records on stdout
    for rec in records:
        assert KEYS <= set(rec)
        assert rec['value'] == records[0]['value']  # every line carries the same headline
    return records


@pytest.mark.parametrize('nproc,model', [(1, 'unet'), (2, 'unet'), (2, 'amoebanet'),
                                         (1, 'resnet'), (4, 'unet'), (8, 'unet'),
                                         (8, 'amoebanet')])
def test_bench_json_contract(nproc, model):
    """The driver's N = 1 / 2 / 4 / 8 invocations (``torch.distributed.run``, one rank per
    GPU; here gloo CPU ranks and the tiny model variants): every section runs at every N,
    the 8-rank run included, and reports its wall time."""
    rec = _run(nproc, '--model', model)
    assert KEYS <= set(rec)
    assert rec['n_gpus'] == nproc and rec['steps'] == 1 and rec['warmup'] == 1
    assert rec['value'] > 0 and rec['higher_is_better'] is True
    assert rec['config']['global_batch'] == 4
    assert rec['config']['parallelism'] == f'pp{nproc}'
    assert 'TINY' in rec['metric'] and rec['vs_baseline'] is None
    if model == 'resnet':
        assert rec['metric'].startswith('ResNet-101')
        assert rec['config']['checkpoint'] == 'except_last'
    # value is the whole-job aggregate: batch * steps / elapsed
    assert rec['value'] == pytest.approx(4 * 1000 / rec['ms_per_step'], rel=1e-2)
    if model == 'unet' and nproc == 1:
        # the public single-process GPipe API on the headline experiment
        assert rec['gpipe']['value'] > 0 and rec['gpipe']['chunks'] == 2
        assert rec['gpipe']['vs_pipeline_stage'] == pytest.approx(
            rec['gpipe']['value'] / rec['value'], rel=1e-2)
    if model == 'unet':
        # same-box speed-up denominator and the AmoebaNet section ride along
        assert rec['baseline']['value'] > 0 and rec['speedup_vs_baseline'] > 0
        assert rec['speedup_vs_baseline'] == pytest.approx(
            rec['value'] / rec['baseline_samples_per_sec'], rel=1e-2)
        amoeba = rec['amoebanet']
        assert amoeba['value'] > 0 and amoeba['steps'] == 1
        if nproc == 2:
            assert amoeba['n2m1']['chunks'] == 1 and amoeba['speedup_vs_n2m1'] > 0
        # ResNet-101 section (tiny stand-in): pipeline-1 at N=1, config #2's shape at N=2,
        # the reference's pipeline-4 / -8 at N=4 / 8
        res = rec['resnet101']
        assert res['value'] > 0 and res['checkpoint'] == ('always' if nproc == 2
                                                           else 'except_last')
        want = {'headline', 'baseline', 'amoebanet', 'resnet'}
        # (the tiny variant's tuned balance is its reference one: no 'tuned' section)
        want |= {'gpipe'} if nproc == 1 else {'graph_cells'}
        want |= {'striped'} if nproc >= 3 else set()
        assert set(rec['section_s']) == want
        # with its own no-GPipe denominator (the reference's ResNet baseline, B=118)
        assert res['baseline']['value'] > 0
        assert res['speedup_vs_baseline'] == pytest.approx(
            res['value'] / res['baseline']['value'], rel=1e-2)
    if nproc > 1:
        ranks = rec['per_rank']
        assert [r['rank'] for r in ranks] == list(range(nproc))
        for r in ranks:
            assert r['step_ms'] > 0 and r['busy_ms'] <= r['step_ms'] + 1e-6
            assert min(r['fwd_wait_ms'], r['bwd_wait_ms'], r['fill_ms'], r['drain_ms']) >= 0
            assert r['host_enqueue_ms'] > 0
        # rank 1 waits for rank 0's activations, rank 0 for rank 1's gradients
        assert ranks[1]['fwd_wait_ms'] > 0 and ranks[0]['bwd_wait_ms'] > 0


def test_bench_headline_printed_before_the_sections_eight_ranks():
    """At N=8 the first line is the headline alone (the reference balance on the plain
    eager engine: no stripes, no captured cells), printed before any section runs; each
    later line adds one section."""
    records = _run_lines(8, '--model', 'unet', '--sections', 'baseline,amoebanet,striped')
    first = records[0]
    assert set(first['section_s']) == {'headline'}
    assert 'baseline' not in first and 'amoebanet' not in first and 'striped' not in first
    assert first['config']['striped_routes'] == {} and first['config']['graph_cells'] is False
    assert first['config']['balance_source'] == 'ref'
    assert [set(r['section_s']) for r in records[1:]] == [
        {'headline', 'baseline'}, {'headline', 'baseline', 'amoebanet'},
        {'headline', 'baseline', 'amoebanet', 'striped'}]


def test_bench_failed_optional_section_keeps_the_run():
    """N > 1: an opt-in variant that raises on every rank (here injected into ``striped``)
    is recorded under its key, the sections after it are skipped, the earlier lines stand
    and the ranks exit cleanly instead of tearing down communicators mid-exchange."""
    records = _run_lines(3, '--model', 'unet', '--sections', 'baseline,striped,graph_cells',
                         env_extra={'TGPIPE_BENCH_FAIL': 'striped'})
    last = records[-1]
    assert 'failure injected' in last['striped']['error']
    assert 'amoebanet_graph_cells' not in last
    assert last['baseline']['value'] > 0 and last['value'] == records[0]['value']
    assert set(last['section_s']) == {'headline', 'baseline', 'striped'}


def test_bench_striped_eight_ranks():
    """The ``striped`` section at 8 ranks with a threshold every tiny message clears: the
    headline U-Net's routes are planned after the first warm-up step (an extra untimed
    step), relayed in the timed step, and reported under their own key."""
    rec = _run(8, '--model', 'unet', '--stripe-mb', '0.000001', '--sections', 'striped')
    assert rec['config']['striped_routes'] == {}  # the headline stays direct
    routes = rec['striped']['striped_routes']
    assert routes, rec['striped']
    for route, relays in routes.items():
        src, dst = map(int, route.split('->'))
        assert relays and not {src, dst} & set(relays)
    assert rec['striped']['value'] > 0


def test_bench_headline_uses_reference_balance_and_reports_tuned():
    """N > 1: the headline runs the reference balance; --also-tuned adds the MI355X one."""
    rec = _run(2, '--model', 'unet', '--also-tuned', 'yes')
    assert rec['config']['balance_source'] == 'ref'
    tuned = rec['tuned']
    assert tuned is not None and tuned['value'] > 0 and sum(tuned['balance']) == sum(
        rec['config']['balance'])


def test_bench_reference_balance_tables():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.UNET_EXPERIMENTS[8]['balance'] == [16, 27, 31, 44, 22, 57, 27, 17]
    assert bench.UNET_EXPERIMENTS[4]['balance'] == [30, 66, 84, 61]
    assert bench.UNET_EXPERIMENTS[2]['balance'] == [104, 137]
    assert bench.AMOEBA_EXPERIMENTS[8]['balance'] == [2, 2, 2, 3, 3, 4, 4, 4]
