"""Multi-process pipeline (PipelineStage / DistributedGPipe) on gloo CPU ranks.

The same code path runs over RCCL on MI355X; here every rank is a CPU process.
"""
import pytest
import torch
from torch import nn
import torch.nn.functional as F

from tests.distributed.mp_util import run
from torchgpipe_amd.skip import Namespace, pop, skippable, stash


@skippable(stash=['skip'])
class Stash(nn.Module):
    def forward(self, x):
        yield stash('skip', x)
        return x


@skippable(pop=['skip'])
class PopAdd(nn.Module):
    def forward(self, x):
        s = yield pop('skip')
        return x + s


class Split(nn.Module):
    def forward(self, x):
        return x, x * 0.5


class Merge(nn.Module):
    def __init__(self):
        super().__init__()
        self.fc = nn.Linear(8, 8)

    def forward(self, xy):
        x, y = xy
        return self.fc(x) + y


def build(dropout=0.0):
    torch.manual_seed(1234)
    ns = Namespace()
    return nn.Sequential(
        nn.Linear(4, 8), Stash().isolate(ns), nn.Tanh(),       # 0-2
        nn.Linear(8, 8), Split(),                               # 3-4  (tuple boundary)
        Merge(), nn.Dropout(dropout),                           # 5-6
        PopAdd().isolate(ns), nn.Linear(8, 2))                  # 7-8


BALANCE = [3, 2, 4]
X = torch.randn(12, 4, generator=torch.Generator().manual_seed(5))
T = torch.randn(12, 2, generator=torch.Generator().manual_seed(6))


def reference_grads():
    model = build()
    loss = F.mse_loss(model(X), T)
    loss.backward()
    grads = [p.grad.clone() for p in model.parameters()]
    return grads, loss.item()


def _stage_worker(rank, world, checkpoint, chunks, links, dropout):
    from torchgpipe_amd.parallel import PipelineStage
    stage = PipelineStage(build(dropout), BALANCE, chunks=chunks, checkpoint=checkpoint,
                          links=links)
    torch.manual_seed(100 + rank)
    loss = stage.train_step(X if rank == 0 else None, T if rank == world - 1 else None,
                            F.mse_loss)
    return {'grads': [p.grad.clone() for p in stage.parameters()],
            'loss': None if loss is None else loss.item(),
            'in_skips': len(stage.in_skips), 'out_skips': len(stage.out_skips)}


@pytest.mark.parametrize('checkpoint', ['always', 'except_last', 'never'])
def test_stage_gradients_match_single_process(tmp_path, checkpoint):
    results = run(_stage_worker, 3, tmp_path, checkpoint, 4, None, 0.0)
    grads, loss = reference_grads()
    got = [g for r in results for g in r['grads']]
    assert len(got) == len(grads)
    for a, b in zip(got, grads):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    assert abs(results[-1]['loss'] - loss) < 1e-6
    # rank 0 stashes for rank 2; rank 2 pops it
    assert results[0]['out_skips'] == 1 and results[2]['in_skips'] == 1


def test_stage_with_dedicated_link_groups(tmp_path):
    results = run(_stage_worker, 3, tmp_path, 'except_last', 3, True, 0.0)
    grads, _ = reference_grads()
    for a, b in zip([g for r in results for g in r['grads']], grads):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def test_stage_dropout_recompute_replays_rng(tmp_path):
    never = run(_stage_worker, 3, tmp_path / 'never', 'never', 4, None, 0.5)
    always = run(_stage_worker, 3, tmp_path / 'always', 'always', 4, None, 0.5)
    for rn, ra in zip(never, always):
        for a, b in zip(rn['grads'], ra['grads']):
            torch.testing.assert_close(a, b)


def _api_worker(rank, world):
    from torchgpipe_amd.distributed import DistributedGPipe
    workers = {r: f'worker{r}' for r in range(world)}
    model = DistributedGPipe(build(), rank, workers, BALANCE, 4)
    outputs = model.forward(X if rank == 0 else None)
    if rank == world - 1:
        losses = [F.mse_loss(o, t) * (len(t) / len(T)) for o, t in zip(outputs, T.chunk(4))]
        model.backward(losses)
    else:
        model.backward(None)
    return [p.grad.clone() for p in model.parameters()]


def test_distributed_gpipe_api(tmp_path):
    results = run(_api_worker, 3, tmp_path)
    grads, _ = reference_grads()
    for a, b in zip([g for r in results for g in r], grads):
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)


def _loader_worker(rank, world):
    from torchgpipe_amd.distributed import DistributedGPipeDataLoader
    data = [(torch.full((2, 3), float(i)), torch.full((2,), float(i) + 0.5)) for i in range(3)]
    loader = DistributedGPipeDataLoader(data if rank == 0 else None, rank, chunks=2,
                                        num_iterations=3, last_stage=rank == world - 1,
                                        last_stage_name=f'worker{world - 1}')
    out = []
    for x, t in loader:
        out.append((None if x is None else x.clone(), None if t is None else t.clone()))
    return out


def test_data_loader_ships_targets_to_last_stage(tmp_path):
    results = run(_loader_worker, 3, tmp_path)
    assert [x[0, 0].item() for x, t in results[0]] == [0.0, 1.0, 2.0]
    assert all(t is None for _, t in results[0])
    assert all(x is None and t is None for x, t in results[1])
    assert [t[0].item() for x, t in results[2]] == [0.5, 1.5, 2.5]


def _eval_worker(rank, world):
    from torchgpipe_amd.parallel import PipelineStage
    stage = PipelineStage(build(), BALANCE, chunks=3)
    stage.eval()
    with torch.no_grad():
        outs = stage.forward(X if rank == 0 else None)
    return outs


def test_eval_forward_matches_plain_model(tmp_path):
    results = run(_eval_worker, 3, tmp_path)
    model = build().eval()
    with torch.no_grad():
        want = model(X)
    torch.testing.assert_close(torch.cat(results[-1]), want)


def build_unet():
    from torchgpipe_amd.models import unet
    torch.manual_seed(7)
    model = unet(depth=3, num_convs=1, base_channels=4, input_channels=3, output_channels=1)
    for m in model.modules():  # deterministic: compare against the plain model
        if isinstance(getattr(m, 'p', None), float):
            m.p = 0.0
    return model


UX = torch.rand(6, 3, 16, 16, generator=torch.Generator().manual_seed(8))
UT = torch.rand(6, 1, 16, 16, generator=torch.Generator().manual_seed(9))


def _unet_worker(rank, world, balance, checkpoint):
    from torchgpipe_amd.parallel import PipelineStage
    stage = PipelineStage(build_unet(), balance, chunks=3, checkpoint=checkpoint)
    for _ in range(2):  # second step runs on cached message metadata
        for p in stage.parameters():
            p.grad = None
        loss = stage.train_step(UX if rank == 0 else None, UT if rank == world - 1 else None,
                                F.binary_cross_entropy_with_logits)
    return {'grads': [p.grad.clone() for p in stage.parameters()],
            'loss': None if loss is None else loss.item(),
            'skip_dsts': sorted({d for d, _ in stage.out_skips}),
            'skip_srcs': sorted({s for s, _ in stage.in_skips})}


@pytest.mark.parametrize('checkpoint', ['except_last', 'never'])
def test_unet_skips_fan_out_to_several_ranks(tmp_path, checkpoint):
    """Rank 0 stashes skips popped by two different ranks and receives skip
    gradients back from both: every (kind, micro-batch, src, dst) message has
    its own metadata entry."""
    model = build_unet()
    balance = [17, 9, 6, 9]
    assert sum(balance) == len(model)
    results = run(_unet_worker, 4, tmp_path, balance, checkpoint)
    assert len(results[0]['skip_dsts']) >= 2, results[0]['skip_dsts']
    loss = F.binary_cross_entropy_with_logits(model(UX), UT)
    loss.backward()
    want = [p.grad for p in model.parameters()]
    got = [g for r in results for g in r['grads']]
    assert len(got) == len(want)
    for a, b in zip(got, want):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)
    assert results[-1]['loss'] == pytest.approx(loss.item(), rel=1e-5)


# -- gradient parity of U-Net / AmoebaNet against one process (same harness as RCCL) ------

from tests.distributed import parity  # noqa: E402


@pytest.mark.parametrize('world', [2, 4])
@pytest.mark.parametrize('kind', parity.MODELS)
def test_model_gradients_match_one_process(tmp_path, kind, world):
    """Every rank's gradients and the loss equal the one-process run (gloo twin of
    tests/distributed/test_rccl_multigpu.py)."""
    chunks = 3
    results = run(parity.stage_worker, world, tmp_path, kind, chunks, 'except_last', 'cpu')
    grads, loss = parity.reference(kind, torch.device('cpu'), chunks)
    parity.assert_parity(results, grads, loss, rel=1e-5)
    if kind == 'unet':
        assert any(r['skip_peers'] for r in results)


@pytest.mark.parametrize('kind', ['unet-p8', 'amoebanet-p8'])
def test_reference_eight_partition_balances_match_one_process(tmp_path, kind):
    """The first 8-GPU run's topology, rehearsed on 8 gloo ranks: U-Net(5,5) with all 241
    layers at the reference's pipeline-8 balance [16, 27, 31, 44, 22, 57, 27, 17] -- its
    four long skips fan out across ranks, so ``connect()`` orders 8-way links -- and
    AmoebaNet-D(18) with all 24 layers at the n8 balance [2, 2, 2, 3, 3, 4, 4, 4] ((x, skip)
    tuple boundaries), at tiny widths.  Every gradient and the loss equal one process, in
    float64: at these widths and 2-image micro-batches the fp32 gradients of the first
    layers differ from fp64 by 25 % (AmoebaNet) under any summation order, so fp32 parity
    would only measure rounding."""
    import time
    chunks = 3
    t0 = time.time()
    results = run(parity.stage_worker, 8, tmp_path, kind, chunks, 'except_last', 'cpu',
                  {'dtype': torch.float64})
    print(f'{kind}: 8 ranks in {time.time() - t0:.1f} s')
    grads, loss = parity.reference(kind, torch.device('cpu'), chunks, dtype=torch.float64)
    parity.assert_parity(results, grads, loss, rel=1e-9)
    if kind == 'unet-p8':
        # the long skips really cross ranks: several stashing and popping ranks
        assert sum(1 for r in results if r['skip_peers']) >= 4, [r['skip_peers'] for r in results]


@pytest.mark.parametrize('kind', ['unet-p8', 'amoebanet-p8'])
def test_striped_transfers_match_one_process(tmp_path, kind):
    """Multi-path transfers (``parallel/stripes.py``) on the 8-rank topologies: with a
    1-byte threshold every route of one message kind is striped over idle ranks.  Step 1
    records, step 2 plans and runs striped, step 3 runs striped again (relay rings reused);
    the gradients equal one process in float64, and the plan really relays."""
    chunks = 3
    results = run(parity.stage_worker, 8, tmp_path, kind, chunks, 'except_last', 'cpu',
                  {'dtype': torch.float64, 'stripes': 1, 'steps': 3})
    grads, loss = parity.reference(kind, torch.device('cpu'), chunks, dtype=torch.float64)
    parity.assert_parity(results, grads, loss, rel=1e-9)
    plans = [r['stripes'] for r in results]
    assert all(p == plans[0] for p in plans), plans  # every rank planned alike
    print(kind, 'striped routes:', plans[0])
    assert plans[0], 'nothing striped'
    jobs = [j for r in results for j in r['relay_jobs']]
    assert jobs and all(j in plans[0] for j in jobs), (jobs, plans[0])
    # a relay never relays a route it is an end of, nor over a link the pipeline uses
    for rank, r in enumerate(results):
        for src, dst in r['relay_jobs']:
            assert rank not in (src, dst)
            assert rank in plans[0][(src, dst)]


@pytest.mark.parametrize('kind,world,options', [
    ('unet', 2, dict(backward_thread=True, steps=3)),
    ('amoebanet', 2, dict(backward_thread=True, checkpoint_mode='always', steps=3)),
    ('unet-p8', 8, dict(backward_thread=True, dtype=torch.float64, stripes=1, steps=3)),
])
def test_backward_thread_matches_one_process(tmp_path, kind, world, options):
    """``backward_thread``: each micro-batch's backward issued from a helper thread while
    the main thread recomputes the next one and posts its receives; gradients and loss
    equal one process (with multi-path transfers too at 8 ranks)."""
    options = dict(options)
    checkpoint = options.pop('checkpoint_mode', 'except_last')
    results = run(parity.stage_worker, world, tmp_path, kind, 3, checkpoint, 'cpu', options)
    dtype = options.get('dtype')
    grads, loss = parity.reference(kind, torch.device('cpu'), 3, dtype=dtype)
    parity.assert_parity(results, grads, loss, rel=1e-9 if dtype == torch.float64 else 1e-5)


# -- failure detection: a dead or mis-ordered peer raises within the timeout --------------

def _dead_peer_worker(rank, world):
    import time
    from torchgpipe_amd.parallel import PipelineStage
    from torchgpipe_amd.parallel.p2p import PipelineTimeout
    stage = PipelineStage(build(), BALANCE, chunks=2, timeout=2.0)
    # (the rendezvous store, not the gloo pairs, orders the exits: rank 0 hosts it and
    # leaves last; the others stay until rank 1 has timed out)
    store = torch.distributed.distributed_c10d._get_default_store()
    deadline = time.monotonic() + 60

    def leave() -> None:
        while store.add('dead_timed_out', 0) < 1 and time.monotonic() < deadline:
            time.sleep(0.05)
        store.add('dead_left', 1)
        while rank == 0 and store.add('dead_left', 0) < world and time.monotonic() < deadline:
            time.sleep(0.05)

    if rank != 1:
        leave()  # rank 0 never sends; rank 2 idles too
        return {'raised': None, 'elapsed': 0.0}
    start = time.monotonic()
    try:
        stage.forward(None)
    except PipelineTimeout as exc:
        elapsed = time.monotonic() - start
        store.add('dead_timed_out', 1)
        leave()
        return {'raised': type(exc).__name__, 'elapsed': elapsed, 'msg': str(exc)}
    return {'raised': None, 'elapsed': time.monotonic() - start}


def test_dead_peer_raises_pipeline_timeout(tmp_path):
    results = run(_dead_peer_worker, 3, tmp_path, barrier=False)
    assert results[1]['raised'] == 'PipelineTimeout', results[1]
    assert results[1]["elapsed"] < 10.0, results[1]
    assert 'rank 0' in results[1]['msg']


def _misordered_worker(rank, world):
    import time
    from torchgpipe_amd.parallel.p2p import P2P, PipelineTimeout
    p2p = P2P(torch.device('cpu'), timeout=2.0)
    start = time.monotonic()
    try:
        # Both ranks receive first: the classic mis-ordered exchange that hangs forever
        # under the reference's blocking mailboxes.
        p2p.recv(1 - rank, ('act', 0)).wait()
    except PipelineTimeout as exc:
        elapsed = time.monotonic() - start
        # stay connected until the peer has timed out too (counted on the rendezvous
        # store, not the gloo pair): exiting first would close the pair and turn the
        # peer's timeout into a connection error.  Rank 0 hosts the store, so it leaves
        # last.
        store = torch.distributed.distributed_c10d._get_default_store()
        store.add('misordered_timed_out', 1)
        deadline = time.monotonic() + 60
        while store.add('misordered_timed_out', 0) < world and time.monotonic() < deadline:
            time.sleep(0.05)
        store.add('misordered_left', 1)
        while rank == 0 and store.add('misordered_left', 0) < world and \
                time.monotonic() < deadline:
            time.sleep(0.05)
        return {'raised': type(exc).__name__, 'elapsed': elapsed, 'msg': str(exc)}
    return {'raised': None, 'elapsed': time.monotonic() - start}


def test_misordered_exchange_raises_pipeline_timeout(tmp_path):
    results = run(_misordered_worker, 2, tmp_path, barrier=False)
    for r in results:
        assert r['raised'] == 'PipelineTimeout', r
        assert r["elapsed"] < 10.0, r
        assert "'act'" in r['msg']


@pytest.mark.parametrize('kind,options', [
    ('unet', dict(overlap_recompute=True, overlap_forward=True, graph_cells=True, steps=3)),
    ('amoebanet', dict(cell_streams=True, graph_cells=True, steps=3)),
])
def test_bench_options_cpu_twin(tmp_path, kind, options):
    """CPU/gloo twin of tests/distributed/test_rccl_multigpu.py::
    test_rccl_bench_options_match_single_gpu: the GPU-only options are accepted and the
    stage runs its eager schedule."""
    results = run(parity.stage_worker, 2, tmp_path, kind, 3, 'except_last', 'cpu', options)
    grads, loss = parity.reference(kind, torch.device('cpu'), 3)
    parity.assert_parity(results, grads, loss, rel=1e-5)
    assert all(r['phases'] == ['eager'] * 3 for r in results)
