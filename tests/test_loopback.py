"""LoopbackP2P: one stage of a multi-rank pipeline in one process (stage emulation).

The stand-in transport must feed a PipelineStage exactly the messages a real pipeline
would: the boundary activations / skips of its rank, gradients shaped like what it sent,
and nothing for ranks without neighbours -- so ``benchmarks/stage_harness.py`` times the
real engine.  CPU: every rank of a U-Net (skips fanning out) and an AmoebaNet ((x, skip)
tuple boundaries) steps, and the first rank's gradients equal a plain run of its layers
with the same output gradients.
"""
import copy

import pytest
import torch
import torch.nn.functional as F

from torchgpipe_amd.microbatch import Batch
from torchgpipe_amd.parallel import PipelineStage
from torchgpipe_amd.parallel.loopback import LoopbackP2P
from torchgpipe_amd.parallel.stage import signature_of
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker


def _model(kind):
    torch.manual_seed(0)
    if kind == 'unet':
        from torchgpipe_amd.models import unet
        model = unet(depth=3, num_convs=1, base_channels=4, input_channels=3, output_channels=1)
        return model, (3, 16, 16)
    from torchgpipe_amd.models import amoebanetd
    return amoebanetd(num_classes=10, num_layers=3, num_filters=8), (3, 224, 224)


def _stage(kind, balance, k, chunks=2, batch=4):
    model, shape = _model(kind)
    layers = list(model)
    lo = sum(balance[:k])
    tracker = SkipTracker()
    with torch.no_grad(), use_skip_tracker(tracker):
        b = Batch(torch.rand(batch // chunks, *shape))
        for layer in layers[:lo]:
            b = b.call(layer)
    transport = LoopbackP2P(torch.device('cpu'), list(b), b.atomic, {})
    stage = PipelineStage(model, balance, rank=k, chunks=chunks, transport=transport)
    skips = {}
    for src, key in stage.in_skips:
        skips.setdefault(src, []).append(tracker.tensors[key])
    transport.skips = skips
    return stage, transport, shape


@pytest.mark.parametrize('kind,balance', [('unet', [11, 8, 7]), ('amoebanet', [3, 4, 2])])
def test_every_rank_steps_on_the_loopback(kind, balance):
    balance = list(balance)
    model, _ = _model(kind)
    balance[-1] = len(model) - sum(balance[:-1])
    for k in range(len(balance)):
        stage, transport, shape = _stage(kind, balance, k)
        sig = signature_of(torch.empty(4, *shape))
        x = torch.rand(4, *shape) if stage.is_first else None
        if kind == 'unet':
            t = torch.rand(4, 1, *shape[1:]) if stage.is_last else None
            loss_fn = F.binary_cross_entropy_with_logits
        else:
            t = torch.randint(10, (4,)) if stage.is_last else None
            loss_fn = F.cross_entropy
        for _ in range(2):
            for p in stage.parameters():
                p.grad = None
            stage.train_step(x, t, loss_fn, signature=sig)
        assert all(p.grad is not None for p in stage.parameters()), k
        # what it sent downstream / to the skip pop ranks is what it would send for real
        kinds = {key[0] for key in transport._sent}
        if not stage.is_last:
            assert 'act' in kinds
        if stage.out_skips:
            assert 'skip' in kinds
        if not stage.is_first:
            assert 'gact' in kinds


def test_first_rank_gradients_match_its_layers():
    """Rank 0 of 2 on the loopback: its gradients are those of its layers back-propagated
    from the (random) output gradients the transport handed it."""
    kind, balance = 'amoebanet', [3, 6]
    model, _ = _model(kind)
    balance[-1] = len(model) - balance[0]
    stage, transport, shape = _stage(kind, balance, 0)
    ref = copy.deepcopy(stage.partition)
    x = torch.rand(4, *shape)
    stage.train_step(x, None, F.cross_entropy, signature=signature_of(x))
    for i, xc in enumerate(x.chunk(2)):
        out = Batch(ref(xc))
        key = next(key for key in transport._bufs if key[3] == 'gact' and key[4] == i)
        grads = transport._bufs[key]
        ys = [y for y in out if y.requires_grad]
        torch.autograd.backward(ys, grads)
    for (name, pa), pb in zip(ref.named_parameters(), stage.parameters()):
        torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-5, atol=1e-6, msg=name)


def test_uneven_micro_batches_on_the_last_rank():
    """A mini-batch that does not split evenly (7 images in 3 micro-batches: 3, 3, 1, as
    ResNet-101's B=25000 in 1667): with the micro-batch sizes the loopback trims its
    templates, so the last rank's outputs line up with the target's chunks."""
    kind, balance = 'amoebanet', [3, 6]
    model, shape = _model(kind)
    balance[-1] = len(model) - balance[0]
    layers = list(model)
    tracker = SkipTracker()
    with torch.no_grad(), use_skip_tracker(tracker):
        b = Batch(torch.rand(3, *shape))
        for layer in layers[:balance[0]]:
            b = b.call(layer)
    sizes = [len(c) for c in torch.empty(7, 0).chunk(3)]
    assert sizes == [3, 3, 1]
    transport = LoopbackP2P(torch.device('cpu'), list(b), b.atomic, {}, sizes)
    stage = PipelineStage(model, balance, rank=1, chunks=3, transport=transport)
    loss = stage.train_step(None, torch.randint(10, (7,)), F.cross_entropy,
                            signature=signature_of(torch.empty(7, *shape)))
    assert loss is not None and torch.isfinite(loss)
    assert all(p.grad is not None for p in stage.parameters())
