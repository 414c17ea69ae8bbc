"""Multi-rank pipelines with intra-rank stream overlap, rehearsed on ONE GPU.

Two or three ranks share ``cuda:0`` and exchange host-staged messages over gloo, so
every stream decision of :class:`~torchgpipe_amd.parallel.PipelineStage` runs on a real
device: forward lanes (micro-batches alternating between two streams, their sends
leaving from the lane), the recompute lane beside the gradient receive, backward
ordering across lanes (the fused ops add into ``.grad`` outside autograd) and
AmoebaNet's two-stream cells.  Gradients of every rank and the loss are checked
against the whole model on one GPU with the same micro-batching
(``tests/distributed/parity.py``).  These are the schedules ``bench.py`` runs on
multi-GPU nodes over RCCL.
"""
import pytest
import torch

from tests.distributed import parity
from tests.distributed.mp_util import run

pytestmark = pytest.mark.gpu

CASES = [
    ('unet', 'except_last', dict(overlap_recompute=True, overlap_forward=True)),
    ('unet', 'except_last', dict(overlap_forward=True)),
    ('unet', 'never', dict(overlap_forward=True)),
    ('unet', 'always', dict(overlap_recompute=True)),
    ('amoebanet', 'except_last', dict(cell_streams=True)),
    ('amoebanet', 'except_last', dict(cell_streams=True, overlap_recompute=True)),
    # captured cells (parallel/segments.py): warm-up, capture and two replayed steps with
    # the persistent receive buffers, the transfers between graph launches
    ('unet', 'except_last', dict(overlap_recompute=True, overlap_forward=True,
                                 graph_cells=True, steps=5)),
    ('unet', 'always', dict(graph_cells=True, steps=5)),
    ('amoebanet', 'except_last', dict(cell_streams=True, graph_cells=True, steps=5)),
    ('amoebanet', 'always', dict(overlap_recompute=True, graph_cells=True, steps=5)),
    # backward issued from a helper thread while the next micro-batch recomputes
    ('unet', 'except_last', dict(overlap_recompute=True, overlap_forward=True,
                                 backward_thread=True, steps=3)),
    ('amoebanet', 'always', dict(cell_streams=True, backward_thread=True, steps=3)),
]


@pytest.mark.parametrize('kind,checkpoint,options', CASES,
                         ids=[f'{k}-{c}-{"+".join(x for x in o if x != "steps")}'
                              for k, c, o in CASES])
def test_overlapped_stage_matches_one_gpu(tmp_path, kind, checkpoint, options):
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    chunks = 3
    results = run(parity.stage_worker, 2, tmp_path, kind, chunks, checkpoint, 'cuda-shared',
                  options, backend='gloo', timeout=120)
    grads, loss = parity.reference(kind, torch.device('cuda', 0), chunks)
    parity.assert_parity(results, grads, loss, rel=1e-4)
    if options.get('graph_cells'):
        want = ['eager', 'eager', 'capture', 'replay', 'replay']
        assert all(r['phases'] == want for r in results), [r['phases'] for r in results]


@pytest.mark.parametrize('kind,options', [
    ('amoebanet', dict(cell_streams=True, stripes=1, steps=3)),
    # (a 4-rank U-Net's skips leave no idle detour: nothing would be striped)
    ('amoebanet', dict(cell_streams=True, overlap_recompute=True, stripes=1, steps=3)),
])
def test_striped_stage_matches_one_gpu(tmp_path, kind, options):
    """Multi-path transfers (``parallel/stripes.py``) with device tensors: four ranks on
    ``cuda:0``, the 0 -> 1 boundary striped (1-byte threshold) through rank 3 (the one
    idle detour of a 4-stage chain), whose relay threads forward host-staged pieces;
    record, plan, two striped steps.  (RCCL relays run the same chains stream-ordered;
    one GPU cannot host two RCCL ranks.)"""
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    chunks = 3
    results = run(parity.stage_worker, 4, tmp_path, kind, chunks, 'except_last', 'cuda-shared',
                  options, backend='gloo', timeout=120)
    grads, loss = parity.reference(kind, torch.device('cuda', 0), chunks)
    parity.assert_parity(results, grads, loss, rel=1e-4)
    assert results[0]['stripes'], 'nothing striped'
    assert any(r['relay_jobs'] for r in results)
