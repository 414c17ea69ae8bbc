"""Multi-process pipeline over RCCL (one rank per GPU): gradient parity with one GPU.

Same harness as the gloo CPU twin (``test_pipeline_stage.py::
test_model_gradients_match_one_process``): U-Net (long skips fanning out to
several ranks) and AmoebaNet ((x, skip) tuple boundaries), 2 and 4 ranks, every
rank's gradients and the loss against the whole model on ``cuda:0`` with the same
micro-batching.  The HIP kernels are deterministic per micro-batch, so the only
differences are fp32 reduction order in split-K kernels: 1e-4 relative per tensor.
Self-skips when the box has fewer GPUs than ranks.
"""
import pytest
import torch

from tests.distributed import parity
from tests.distributed.mp_util import run

pytestmark = [pytest.mark.gpu, pytest.mark.multigpu]


@pytest.mark.parametrize('world', [2, 4])
@pytest.mark.parametrize('kind', parity.MODELS)
@pytest.mark.parametrize('checkpoint', ['except_last', 'always'])
def test_rccl_pipeline_matches_single_gpu(tmp_path, kind, world, checkpoint):
    """Lazily created per-link communicators: the bench.py configuration."""
    if torch.cuda.device_count() < world:
        pytest.skip(f'needs {world} GPUs')
    chunks = 3
    results = run(parity.stage_worker, world, tmp_path, kind, chunks, checkpoint, 'cuda',
                  backend='nccl-lazy', timeout=120)
    grads, loss = parity.reference(kind, torch.device('cuda', 0), chunks)
    parity.assert_parity(results, grads, loss, rel=1e-4)


# The stream options bench.py turns on at N > 1 (U-Net: forward and recompute lanes;
# AmoebaNet: multi-stream cells), alone and with captured cells: the first RCCL run of a
# multi-GPU node checks the stream-ordered receive waits against every lane layout.
BENCH_OPTIONS = {
    'unet': [dict(overlap_recompute=True, overlap_forward=True),
             dict(overlap_recompute=True, overlap_forward=True, graph_cells=True, steps=5)],
    'amoebanet': [dict(cell_streams=True),
                  dict(cell_streams=True, graph_cells=True, steps=5)],
}
BENCH_CASES = [(kind, world, opts) for kind in parity.MODELS for world in (2, 4)
               for opts in BENCH_OPTIONS[kind]]


@pytest.mark.parametrize('kind,world,options', BENCH_CASES,
                         ids=[f'{k}-{w}-{"+".join(x for x in o if x != "steps")}'
                              for k, w, o in BENCH_CASES])
def test_rccl_bench_options_match_single_gpu(tmp_path, kind, world, options):
    """bench.py's N > 1 stage options over RCCL, lazily created per-link communicators."""
    if torch.cuda.device_count() < world:
        pytest.skip(f'needs {world} GPUs')
    chunks = 3
    results = run(parity.stage_worker, world, tmp_path, kind, chunks, 'except_last', 'cuda',
                  options, backend='nccl-lazy', timeout=120)
    grads, loss = parity.reference(kind, torch.device('cuda', 0), chunks)
    parity.assert_parity(results, grads, loss, rel=1e-4)
    if options.get('graph_cells'):
        assert all(r['phases'][-1] == 'replay' for r in results)


@pytest.mark.parametrize('kind', parity.MODELS)
def test_rccl_eager_communicator_with_link_groups(tmp_path, kind):
    """Eager init (``device_id``): one 2-rank group per pipeline link."""
    world = 4
    if torch.cuda.device_count() < world:
        pytest.skip(f'needs {world} GPUs')
    results = run(parity.stage_worker, world, tmp_path, kind, 3, 'except_last', 'cuda',
                  backend='nccl', timeout=120)
    grads, loss = parity.reference(kind, torch.device('cuda', 0), 3)
    parity.assert_parity(results, grads, loss, rel=1e-4)


@pytest.mark.parametrize('kind,world', [('amoebanet', 4), ('unet-p8', 8)])
def test_rccl_striped_transfers_match_single_gpu(tmp_path, kind, world):
    """Multi-path transfers over RCCL (``parallel/stripes.py``): relay chains stream-ordered
    on each relay's route streams, relay links opened in one sorted order; every route
    of one message kind striped (1-byte threshold), record + plan + two striped steps."""
    if torch.cuda.device_count() < world:
        pytest.skip(f'needs {world} GPUs')
    chunks = 3
    results = run(parity.stage_worker, world, tmp_path, kind, chunks, 'except_last', 'cuda',
                  dict(stripes=1, steps=4), backend='nccl-lazy', timeout=120)
    grads, loss = parity.reference(kind, torch.device('cuda', 0), chunks)
    # (fp32 on the 241-layer U-Net: summation order differs between one and eight GPUs)
    parity.assert_parity(results, grads, loss, rel=1e-4 if world == 4 else 1e-3)
    assert results[0]['stripes'] and any(r['relay_jobs'] for r in results)
