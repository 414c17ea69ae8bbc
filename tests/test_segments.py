"""PipelineStage(graph_cells=True): per-cell hipGraph replay (torchgpipe_amd/parallel/segments.py).

The captured cells must train exactly like the eager schedule: same losses, gradients and
SGD-updated parameters over warm-up, capture and replay steps, with the lanes on or off,
for every checkpoint mode; dropout masks must change every step and the recomputation
must reproduce the forward's masks (checked against an oracle that runs each micro-batch
once, eagerly, under the same device Philox slot values).
"""
import copy

import pytest
import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd.parallel import PipelineStage


def test_cpu_stage_ignores_graph_cells():
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(4, 8), nn.ReLU(), nn.Linear(8, 2))
    a, b = copy.deepcopy(model), copy.deepcopy(model)
    sa = PipelineStage(a, [3], chunks=2)
    sb = PipelineStage(b, [3], chunks=2, graph_cells=True)
    x, y = torch.randn(4, 4), torch.randn(4, 2)
    for _ in range(3):
        assert torch.equal(sa.train_step(x, y, F.mse_loss), sb.train_step(x, y, F.mse_loss))
    assert sb.graph_phase == 'eager'
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa.grad, pb.grad)


def test_graph_cells_option_checks():
    model = nn.Sequential(nn.Linear(4, 4))
    with pytest.raises(ValueError, match='warm-up'):
        PipelineStage(model, [1], graph_cells=True, graph_warmup=0)


def _models(kind):
    from torchgpipe_amd.models import amoebanetd, unet
    torch.manual_seed(0)
    if kind == 'unet':
        base = unet(depth=3, num_convs=2, base_channels=16)
        for m in base.modules():  # deterministic comparison: no dropout here
            if isinstance(getattr(m, 'p', None), float):
                m.p = 0.0
        return base, (3, 64, 64), None
    return amoebanetd(num_classes=10, num_layers=3, num_filters=16), (3, 224, 224), 10


def _batch(kind, shape, classes, gen, dev):
    x = torch.rand(8, *shape, device=dev, generator=gen)
    if classes is None:
        return x, torch.rand(8, 1, 64, 64, device=dev, generator=gen), \
            F.binary_cross_entropy_with_logits
    return x, torch.randint(classes, (8,), device=dev, generator=gen), F.cross_entropy


@pytest.mark.gpu
@pytest.mark.parametrize('kind,checkpoint,lanes', [
    ('unet', 'except_last', True),
    ('unet', 'always', False),
    ('unet', 'never', True),
    ('amoebanet', 'except_last', False),
    ('amoebanet', 'always', True),
])
def test_graph_cells_train_like_eager(kind, checkpoint, lanes):
    dev = torch.device('cuda', 0)
    base, shape, classes = _models(kind)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    opts = dict(overlap_recompute=lanes, overlap_forward=lanes)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint, **opts)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       graph_cells=True, **opts)
    if kind == 'amoebanet' and lanes:
        from torchgpipe_amd.models.amoebanet import set_cell_streams
        set_cell_streams(sa.partition, True)
        set_cell_streams(sb.partition, True)
    oa = torch.optim.SGD(sa.parameters(), lr=0.05)
    ob = torch.optim.SGD(sb.parameters(), lr=0.05)
    gen = torch.Generator(device=dev).manual_seed(5)
    phases = []
    for step in range(5):
        x, y, loss_fn = _batch(kind, shape, classes, gen, dev)
        la = sa.train_step(x, y, loss_fn)
        lb = sb.train_step(x, y, loss_fn)
        phases.append(sb.graph_phase)
        torch.cuda.synchronize()
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
            scale = pa.grad.abs().max().item() + 1e-12
            torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-4, atol=1e-5 * scale,
                                       msg=lambda m: f'step {step} {name}: {m}')
        # Both models continue from the same SGD-updated weights (new values every step:
        # the captured graphs must see them through the in-place refreshed weight
        # transforms).  Stepping each model on its own would let fp32 rounding noise grow
        # chaotically through a few updates of this tiny U-Net (eager with and without
        # lanes drift apart by percents too).
        oa.step()
        ob.step()
        with torch.no_grad():
            for pa, pb in zip(a.parameters(), b.parameters()):
                pb.copy_(pa)
        oa.zero_grad(set_to_none=True)
        ob.zero_grad(set_to_none=True)
    assert phases == ['eager', 'eager', 'capture', 'replay', 'replay']
    # running statistics (AmoebaNet BatchNorm) follow the same updates
    for (name, ba), bb in zip(a.named_buffers(), b.buffers()):
        if ba.is_floating_point():
            torch.testing.assert_close(bb, ba, rtol=1e-4, atol=1e-5, msg=name)


@pytest.mark.gpu
def test_graph_cells_dropout_masks_fresh_and_replayed():
    """U-Net with Dropout2d (p=0.1) in the fused cells: every replayed step draws new
    masks, and the gradients equal an eager oracle run under the very Philox values the
    graphs read (so the recomputation reproduced the forward's masks)."""
    from torchgpipe_amd.models import unet
    from torchgpipe_amd.utils import rng
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = unet(depth=2, num_convs=2, base_channels=16)
    model = copy.deepcopy(base)
    oracle = copy.deepcopy(base).to(dev)
    stage = PipelineStage(model, [len(model)], device=dev, chunks=2, checkpoint='always',
                          graph_cells=True)
    x = torch.rand(4, 3, 32, 32, device=dev)
    y = torch.rand(4, 1, 32, 32, device=dev)
    losses = []
    for step in range(5):
        for p in stage.parameters():
            p.grad = None
        losses.append(stage.train_step(x, y, F.binary_cross_entropy_with_logits).item())
    assert stage.graph_phase == 'replay'
    assert len(set(losses[2:])) == 3, losses  # fresh masks every step
    # oracle: each micro-batch once, with grad, under the slot values of the last step
    slots = stage._segments.slots.clone()
    for p in oracle.parameters():
        p.grad = None
    for i, (xc, yc) in enumerate(zip(x.chunk(2), y.chunk(2))):
        slot = rng.PhiloxSlot(slots[i].clone())
        with rng.slot_scope(slot):
            out = oracle(xc)
        (F.binary_cross_entropy_with_logits(out, yc) * (yc.size(0) / 4.0)).backward()
    for (name, po), pm in zip(oracle.named_parameters(), model.parameters()):
        scale = po.grad.abs().max().item() + 1e-12
        torch.testing.assert_close(pm.grad, po.grad, rtol=1e-4, atol=1e-5 * scale, msg=name)


@pytest.mark.gpu
def test_graph_cells_deferred_batch_norm_commits():
    """DeferredBatchNorm's commit happens inside the last cell's captured forward: the
    running statistics after replayed steps equal the eager stage's."""
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.BatchNorm2d(8), nn.ReLU(),
                         nn.Conv2d(8, 4, 3, padding=1), nn.BatchNorm2d(4), nn.Flatten(),
                         nn.Linear(4 * 8 * 8, 3))
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, deferred_batch_norm=True)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, deferred_batch_norm=True,
                       graph_cells=True)
    gen = torch.Generator(device=dev).manual_seed(3)
    for _ in range(5):
        x = torch.randn(8, 3, 8, 8, device=dev, generator=gen) * 2 + 1
        y = torch.randint(3, (8,), device=dev, generator=gen)
        sa.train_step(x, y, F.cross_entropy)
        sb.train_step(x, y, F.cross_entropy)
    torch.cuda.synchronize()
    assert sb.graph_phase == 'replay'
    for (name, ba), bb in zip(sa.partition.named_buffers(), sb.partition.buffers()):
        if ba.is_floating_point():
            torch.testing.assert_close(bb, ba, rtol=1e-5, atol=1e-6, msg=name)
        else:
            assert torch.equal(bb, ba), name


@pytest.mark.gpu
@pytest.mark.parametrize('graph_warmup', [1, 2])
def test_graph_cells_accumulate_over_train_steps_like_eager(graph_warmup):
    """Two ``train_step`` calls before ``optimizer.step()`` (gradient accumulation) give
    eager's summed gradients in every phase -- including the capture step with a single
    warm-up step, whose captures meet the weight-transform caches empty -- and a parameter
    no backward reaches keeps ``.grad`` None."""
    dev = torch.device('cuda', 0)
    base, shape, classes = _models('unet')
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    # a parameter of a partition's layer that no forward uses
    b[0].register_parameter('unused_weight', nn.Parameter(torch.ones(3, device=dev)))
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, graph_cells=True,
                       graph_warmup=graph_warmup)
    pbs = dict(b.named_parameters())
    gen = torch.Generator(device=dev).manual_seed(7)
    phases = []
    for step in range(5):
        for _ in range(2):
            x, y, loss_fn = _batch('unet', shape, classes, gen, dev)
            sa.train_step(x, y, loss_fn)
            sb.train_step(x, y, loss_fn)
            phases.append(sb.graph_phase)
        torch.cuda.synchronize()
        for name, pa in a.named_parameters():
            pb = pbs[name]
            scale = pa.grad.abs().max().item() + 1e-12
            torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-4, atol=1e-5 * scale,
                                       msg=lambda m: f'step {step} {name}: {m}')
        if 'replay' in phases:
            assert b[0].unused_weight.grad is None
        with torch.no_grad():
            for name, pa in a.named_parameters():
                pa.sub_(0.05 * pa.grad)
                pbs[name].copy_(pa)
        for p in a.parameters():
            p.grad = None
        for p in b.parameters():
            p.grad = None
    assert 'capture' in phases and phases[-1] == 'replay'


@pytest.mark.gpu
def test_graph_cells_zero_grad_in_place_between_steps():
    """``zero_grad(set_to_none=False)`` between steps: the static buffers are zeroed in
    place by the user and the replays accumulate from zero."""
    dev = torch.device('cuda', 0)
    base, shape, classes = _models('unet')
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=2)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=2, graph_cells=True)
    oa = torch.optim.SGD(a.parameters(), lr=0.05)
    ob = torch.optim.SGD(b.parameters(), lr=0.05)
    gen = torch.Generator(device=dev).manual_seed(3)
    for step in range(5):
        x, y, loss_fn = _batch('unet', shape, classes, gen, dev)
        sa.train_step(x, y, loss_fn)
        sb.train_step(x, y, loss_fn)
        torch.cuda.synchronize()
        for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
            scale = pa.grad.abs().max().item() + 1e-12
            torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-4, atol=1e-5 * scale,
                                       msg=lambda m: f'step {step} {name}: {m}')
        oa.step()
        with torch.no_grad():
            for pa, pb in zip(a.parameters(), b.parameters()):
                pb.copy_(pa)
        oa.zero_grad(set_to_none=False)
        ob.zero_grad(set_to_none=False)
    assert sb.graph_phase == 'replay'


def test_graph_cells_reject_cumulative_deferred_batch_norm():
    from torchgpipe_amd.batchnorm import DeferredBatchNorm
    model = nn.Sequential(nn.Conv2d(3, 4, 1), DeferredBatchNorm(4, momentum=None, chunks=2))
    with pytest.raises(ValueError, match='momentum=None'):
        PipelineStage(model, [2], chunks=2, graph_cells=True)
