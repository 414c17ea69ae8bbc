"""Gradient-parity harness of the multi-process pipeline against one process.

The same worker runs on gloo CPU ranks (every CPU test run) and on RCCL with one
GPU per rank (``tests/distributed/test_rccl_multigpu.py``).  The oracle is the
unpartitioned model run in one process on one device with the *same
micro-batching*: the per-micro-batch losses, weighted by micro-batch size, are
back-propagated one by one.  That is exactly GPipe's semantics (BatchNorm sees
micro-batch statistics), so every parameter gradient of every rank and the
loss must match the oracle.  Models run with dropout disabled (``p = 0``) so no
RNG stream has to line up across processes.
"""
import torch
from torch import nn
import torch.nn.functional as F

MODELS = ('unet', 'amoebanet')


def build(kind: str) -> nn.Sequential:
    """``unet`` / ``amoebanet``: small models for 2-4 ranks.  ``unet-p8`` / ``amoebanet-p8``:
    the benchmark architectures themselves -- U-Net(5,5) with all 241 layers (and all four
    long skips), AmoebaNet-D(18) with all 24 layers -- at tiny widths, for the reference's
    8-partition balances."""
    torch.manual_seed(7)
    if kind == 'unet':
        from torchgpipe_amd.models import unet
        model = unet(depth=3, num_convs=1, base_channels=8, input_channels=3, output_channels=1)
    elif kind == 'unet-p8':
        from torchgpipe_amd.models import unet
        model = unet(depth=5, num_convs=5, base_channels=2, input_channels=3, output_channels=1)
    elif kind == 'amoebanet':
        from torchgpipe_amd.models import amoebanetd
        model = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    elif kind == 'amoebanet-p8':
        from torchgpipe_amd.models import amoebanetd
        model = amoebanetd(num_classes=10, num_layers=18, num_filters=16)
    else:
        raise ValueError(kind)
    for m in model.modules():
        if isinstance(getattr(m, 'p', None), float):
            m.p = 0.0
    return model


def data(kind: str, device: torch.device):
    gen = torch.Generator().manual_seed(11)
    if kind.startswith('unet'):
        side = 64 if kind == 'unet-p8' else 16  # five 2x poolings: a 2x2 bottom plane
        x = torch.rand(6, 3, side, side, generator=gen)
        t = torch.rand(6, 1, side, side, generator=gen)
    else:
        x = torch.rand(6, 3, 224, 224, generator=gen)
        t = torch.randint(10, (6,), generator=gen)
    return x.to(device), t.to(device)


def loss_fn(kind: str):
    return F.binary_cross_entropy_with_logits if kind.startswith('unet') else F.cross_entropy


def balance(kind: str, world: int) -> list:
    """Splits that put skips and tuple boundaries across ranks."""
    n = len(build(kind))
    table = {
        ('unet', 2): [11, n - 11],          # skips of the two top levels cross ranks
        ('unet', 4): [8, 10, 6, n - 24],     # rank 0 stashes for two different ranks
        ('amoebanet', 2): [3, n - 3],        # (x, skip) tuple boundary
        ('amoebanet', 4): [2, 2, 2, n - 6],
        # the reference's 8-partition benchmark balances (benchmarks/unet-speed/main.py:23-68,
        # benchmarks/amoebanetd-speed/main.py:35-96)
        ('unet-p8', 8): [16, 27, 31, 44, 22, 57, 27, 17],
        ('amoebanet-p8', 8): [2, 2, 2, 3, 3, 4, 4, 4],
    }
    return table[(kind, world)]


def _cast(x: torch.Tensor, dtype) -> torch.Tensor:
    return x.to(dtype) if dtype is not None and x.is_floating_point() else x


def reference(kind: str, device: torch.device, chunks: int, dtype=None):
    """Gradients and loss of the whole model on one device, same micro-batching
    (``dtype``: e.g. float64 for the deep tiny-width models, whose fp32 gradients differ
    from fp64 by percents under any summation order)."""
    model = build(kind).to(device=device, dtype=dtype)
    x, t = (_cast(v, dtype) for v in data(kind, device))
    fn = loss_fn(kind)
    total = float(x.size(0))
    loss_sum = 0.0
    pairs = list(zip(x.chunk(chunks), t.chunk(chunks)))
    outputs = [model(xc) for xc, _ in pairs]
    for out, (_, tc) in reversed(list(zip(outputs, pairs))):
        loss = fn(out, tc) * (tc.size(0) / total)
        loss.backward()
        loss_sum += loss.item()
    return [p.grad.detach().cpu().clone() for p in model.parameters()], loss_sum


def stage_worker(rank: int, world: int, kind: str, chunks: int, checkpoint: str,
                 device_type: str, options: dict = None):
    """One rank: two training steps (the second on cached message metadata), or
    ``options['steps']`` (captured cells: warm-up, capture, replays).

    ``device_type``: 'cpu', 'cuda' (rank r on cuda:r) or 'cuda-shared' (every rank on
    cuda:0, host-staged gloo transport: the one-GPU rehearsal of a multi-rank run, which
    exercises the stage's stream logic -- lanes, two-stream cells -- for real).
    ``options``: extra PipelineStage keywords, plus ``cell_streams`` (AmoebaNet) and
    ``steps``.  Every step computes the same gradients (same data, no optimizer step), so
    the last step's are compared with the oracle.
    """
    from torchgpipe_amd.parallel import PipelineStage
    options = dict(options or {})
    cell_streams = options.pop('cell_streams', False)
    steps = options.pop('steps', 2)
    dtype = options.pop('dtype', None)
    if device_type == 'cuda':
        device = torch.device('cuda', rank)
    elif device_type == 'cuda-shared':
        device = torch.device('cuda', 0)
    else:
        device = torch.device('cpu')
    model = build(kind)
    if dtype is not None:
        model = model.to(dtype)
    stage = PipelineStage(model, balance(kind, world), device=device, chunks=chunks,
                          checkpoint=checkpoint, timeout=60, **options)
    if cell_streams:
        from torchgpipe_amd.models.amoebanet import set_cell_streams
        set_cell_streams(stage.partition, True)
    x, t = (_cast(v, dtype) for v in data(kind, device))
    loss = None
    phases = []
    for _ in range(steps):
        for p in stage.parameters():
            p.grad = None
        loss = stage.train_step(x if stage.is_first else None, t if stage.is_last else None,
                                loss_fn(kind))
        phases.append(stage.graph_phase)
    if device.type == 'cuda':
        torch.cuda.synchronize(device)
    plans = [v for v in stage._stripe_plans.values() if not isinstance(v, (list, str))]
    return {'stripes': dict(plans[0].stripes) if plans else {},
            'relay_jobs': [tuple(j[:2]) for j in plans[0].jobs] if plans else [],
            'grads': [p.grad.detach().cpu().clone() for p in stage.parameters()],
            'loss': None if loss is None else loss.item(),
            'skip_peers': sorted({d for d, _ in stage.out_skips} | {s for s, _ in stage.in_skips}),
            'phases': phases}


def assert_parity(results, want_grads, want_loss, rel: float) -> None:
    got = [g for r in results for g in r['grads']]
    assert len(got) == len(want_grads), (len(got), len(want_grads))
    for i, (a, b) in enumerate(zip(got, want_grads)):
        assert a.shape == b.shape, (i, a.shape, b.shape)
        scale = b.norm().item() + 1e-12
        err = (a.double() - b.double()).norm().item() / scale
        assert err <= rel, f'parameter {i} {tuple(b.shape)}: relative gradient error {err:.3e}'
    assert results[-1]['loss'] is not None
    assert abs(results[-1]['loss'] - want_loss) <= rel * max(1.0, abs(want_loss)), \
        (results[-1]['loss'], want_loss)
