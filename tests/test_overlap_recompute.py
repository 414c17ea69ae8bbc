"""PipelineStage(overlap_recompute=True): the next micro-batch is recomputed on a second
stream while the current one runs backward (torchgpipe_amd/parallel/stage.py)."""
import copy

import pytest
import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd.parallel import PipelineStage


def test_cpu_stage_ignores_the_option():
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(4, 8), nn.ReLU(), nn.Linear(8, 2))
    a, b = copy.deepcopy(model), copy.deepcopy(model)
    sa = PipelineStage(a, [3], chunks=4, checkpoint='always')
    sb = PipelineStage(b, [3], chunks=4, checkpoint='always', overlap_recompute=True)
    x, y = torch.randn(8, 4), torch.randn(8, 2)
    la = sa.train_step(x, y, F.mse_loss)
    lb = sb.train_step(x, y, F.mse_loss)
    assert torch.equal(la, lb)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa.grad, pb.grad)


def _close_grads(a: nn.Module, b: nn.Module) -> None:
    for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert pb.grad is not None, name
        scale = pa.grad.abs().max().item() + 1e-12
        torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-4, atol=1e-5 * scale)


@pytest.mark.gpu
@pytest.mark.filterwarnings('error:The AccumulateGrad node')
@pytest.mark.parametrize('model_name,checkpoint,recompute', [
    ('unet', 'except_last', True),
    ('unet', 'always', True),
    ('amoebanet', 'except_last', True),
    # forward lanes alone: the non-checkpointed cells' backward passes run on the two
    # lanes and must still be ordered (fused ops add into .grad outside autograd)
    ('unet', 'except_last', False),
    ('unet', 'never', False),
])
def test_overlapped_recompute_matches_inline(model_name, checkpoint, recompute):
    """Same losses and gradients with the recomputation on two lanes as inline, over three
    steps (U-Net: Philox dropout replayed from the tape on the lane; AmoebaNet: fused
    ops writing .grad from the lanes)."""
    from torchgpipe_amd.models import amoebanetd, unet
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    if model_name == 'unet':
        base = unet(depth=3, num_convs=2, base_channels=16)
        shape, classes = (3, 64, 64), None
    else:
        base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
        shape, classes = (3, 224, 224), 10
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       overlap_recompute=recompute, overlap_forward=True)
    gen = torch.Generator(device=dev).manual_seed(7)
    for _ in range(3):
        x = torch.rand(8, *shape, device=dev, generator=gen)
        if classes is None:
            y = torch.rand(8, 1, 64, 64, device=dev, generator=gen)
            loss_fn = F.binary_cross_entropy_with_logits
        else:
            y = torch.randint(classes, (8,), device=dev, generator=gen)
            loss_fn = F.cross_entropy
        for p in list(a.parameters()) + list(b.parameters()):
            p.grad = None
        # the same Philox pairs for both models' dropout
        state = torch.cuda.get_rng_state(dev)
        la = sa.train_step(x, y, loss_fn)
        torch.cuda.set_rng_state(state, dev)
        lb = sb.train_step(x, y, loss_fn)
        torch.cuda.synchronize()
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        _close_grads(a, b)
        if model_name == 'unet':
            # every U-Net weight gradient (the MIOpen-computed ones of the 8-channel
            # decoder convolutions too) is accumulated by the ops themselves: no
            # AccumulateGrad node, shared by micro-batches of two lanes, ever runs
            assert all(hasattr(p, '_tgpipe_grad_accumulator') for p in b.parameters())


@pytest.mark.gpu
def test_overlap_with_two_stream_cells_matches_plain():
    """The one-GPU bench configuration of AmoebaNet (two-stream cells + recompute lanes)
    against the plain one-stream schedule."""
    from torchgpipe_amd.models import amoebanetd
    from torchgpipe_amd.models.amoebanet import set_cell_streams
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    set_cell_streams(b, True)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last',
                       overlap_recompute=True)
    gen = torch.Generator(device=dev).manual_seed(11)
    for _ in range(3):
        x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
        y = torch.randint(10, (8,), device=dev, generator=gen)
        for p in list(a.parameters()) + list(b.parameters()):
            p.grad = None
        la = sa.train_step(x, y, F.cross_entropy)
        lb = sb.train_step(x, y, F.cross_entropy)
        torch.cuda.synchronize()
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        _close_grads(a, b)


@pytest.mark.gpu
def test_weight_gradient_stream_matches_plain():
    """The fused ops' weight-gradient GEMMs on a side stream (``ops.convbn.
    wgrad_stream_scope`` around the training step, with the recompute lanes):
    the same kernels in the same per-stream order as the plain schedule, so losses,
    gradients and SGD-updated parameters agree over several steps
    (profiles/r2/wgrad_stream_steps.log: bit-identical).  Two-stream cells are left out
    here: autograd sums a node's gradient contributions from the two streams in another
    order (~1e-6), which the tiny model's SGD trajectory then amplifies."""
    from torchgpipe_amd.models import amoebanetd
    from torchgpipe_amd.ops.convbn import wgrad_stream_scope
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last',
                       overlap_recompute=True)
    oa = torch.optim.SGD(sa.parameters(), lr=0.05)
    ob = torch.optim.SGD(sb.parameters(), lr=0.05)
    gen = torch.Generator(device=dev).manual_seed(13)
    for _ in range(3):
        x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
        y = torch.randint(10, (8,), device=dev, generator=gen)
        la = sa.train_step(x, y, F.cross_entropy)
        with wgrad_stream_scope(dev):
            lb = sb.train_step(x, y, F.cross_entropy)
        _close_grads(a, b)
        oa.step()
        ob.step()
        torch.cuda.synchronize()
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        oa.zero_grad(set_to_none=True)
        ob.zero_grad(set_to_none=True)
    for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pb, pa, rtol=1e-5, atol=1e-6, msg=name)


@pytest.mark.parametrize('checkpoint', ['always', 'except_last'])
def test_direct_backward_reaches_a_learnable_loss_head(checkpoint):
    """The last stage's direct backward (through the recomputed graph, not the Checkpoint
    node) still gives a parameter the loss reaches around the stage outputs its gradient,
    as ``direct_backward=False`` and the reference's ``loss.backward()`` do."""
    torch.manual_seed(0)
    model = nn.Sequential(nn.Linear(4, 8), nn.ReLU(), nn.Linear(8, 2))
    a, b = copy.deepcopy(model), copy.deepcopy(model)
    head_a = nn.Parameter(torch.tensor([1.5, -0.5]))
    head_b = nn.Parameter(head_a.detach().clone())
    sa = PipelineStage(a, [3], chunks=4, checkpoint=checkpoint, direct_backward=False)
    sb = PipelineStage(b, [3], chunks=4, checkpoint=checkpoint, direct_backward=True)
    x, y = torch.randn(8, 4), torch.randn(8, 2)
    la = sa.train_step(x, y, lambda o, t: F.mse_loss(o * head_a, t))
    lb = sb.train_step(x, y, lambda o, t: F.mse_loss(o * head_b, t))
    torch.testing.assert_close(la, lb)
    assert head_b.grad is not None
    torch.testing.assert_close(head_b.grad, head_a.grad)
    for pa, pb in zip(a.parameters(), b.parameters()):
        torch.testing.assert_close(pb.grad, pa.grad)


@pytest.mark.gpu
@pytest.mark.parametrize('checkpoint', ['except_last', 'always'])
def test_batchnorm_stage_on_lanes_matches_one_stream(checkpoint):
    """A BatchNorm partition (ResNet) on forward and recompute lanes: its running-statistics
    updates are slotted and folded in order (torchgpipe_amd/runstats.py), so losses,
    gradients, running means / variances and counters agree with the one-stream schedule
    over several steps, the recomputations' second updates included.

    MIOpen's default convolution algorithms (the strided layers) are not bitwise
    deterministic (~1e-6), and at these tiny planes (a 2x2 layer4, 4-image micro-batches)
    that flips a ReLU mask element now and then and moves whole gradients by 1e-2..1e-1 in
    two *identical* one-stream runs (scripts/debug/resnet_determinism.py); the
    deterministic algorithms make both schedules reproducible, so they are compared here."""
    from torchgpipe_amd.models.resnet import build_resnet
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        _bn_lanes_vs_one_stream(build_resnet, checkpoint)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det


def _bn_lanes_vs_one_stream(build_resnet, checkpoint):
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = build_resnet([1, 1, 1, 1], num_classes=10)
    a, b = copy.deepcopy(base).to(dev), copy.deepcopy(base).to(dev)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint,
                       overlap_recompute=False, overlap_forward=False)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       overlap_recompute=True, overlap_forward=True)
    assert sb._forward_lanes() is not None  # BatchNorms no longer pin it to one stream
    gen = torch.Generator(device=dev).manual_seed(5)
    for _ in range(3):
        x = torch.rand(16, 3, 64, 64, device=dev, generator=gen)
        y = torch.randint(10, (16,), device=dev, generator=gen)
        for p in list(a.parameters()) + list(b.parameters()):
            p.grad = None
        la = sa.train_step(x, y, F.cross_entropy)
        lb = sb.train_step(x, y, F.cross_entropy)
        torch.cuda.synchronize()
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        _close_grads(a, b)
        # every gradient, the MIOpen stem's and the classifier's too, was accumulated by
        # the ops on the lanes' own streams, none by an AccumulateGrad node shared across
        # lanes (ops/gradacc.py library_conv2d / linear)
        assert all(hasattr(p, '_tgpipe_grad_accumulator') for p in b.parameters())
    for (name, ba), bb in zip(a.named_buffers(), b.buffers()):
        if name.endswith('num_batches_tracked'):
            assert torch.equal(bb, ba), name
        else:
            torch.testing.assert_close(bb, ba, rtol=1e-5, atol=1e-6, msg=name)


@pytest.mark.gpu
def test_library_layers_accumulate_like_autograd():
    """ops.gradacc.library_conv2d / linear: two backward passes accumulate the same
    gradients as autograd on the plain layers (strided conv with bias, Linear on 3-D input)."""
    from torchgpipe_amd.ops import gradacc
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    conv = nn.Conv2d(3, 8, 7, stride=2, padding=3).to(dev)
    lin = nn.Linear(8, 5).to(dev)
    c2, l2 = copy.deepcopy(conv), copy.deepcopy(lin)
    for _ in range(2):
        x = torch.randn(4, 3, 32, 32, device=dev, requires_grad=True)
        x2 = x.detach().clone().requires_grad_(True)
        y = gradacc.linear(gradacc.library_conv2d(x, conv).mean((2, 3))[:, None, :]
                           .expand(4, 3, 8), lin)
        y2 = l2(c2(x2).mean((2, 3))[:, None, :].expand(4, 3, 8))
        g = torch.randn_like(y)
        y.backward(g)
        y2.backward(g)
        torch.testing.assert_close(x.grad, x2.grad, rtol=1e-5, atol=1e-6)
    for p, q in zip(list(conv.parameters()) + list(lin.parameters()),
                    list(c2.parameters()) + list(l2.parameters())):
        torch.testing.assert_close(p.grad, q.grad, rtol=1e-5, atol=1e-6)
        assert hasattr(p, '_tgpipe_grad_accumulator')
