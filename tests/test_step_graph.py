"""Whole-step hipGraph capture (torchgpipe_amd/parallel/graph.py)."""
import copy

import pytest
import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd.ops.dropout import Dropout2d
from torchgpipe_amd.parallel import PipelineStage, StepGraph
from torchgpipe_amd.parallel.graph import rng_modules
from torchgpipe_amd.utils import rng


def _mlp() -> nn.Sequential:
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(8, 16), nn.ReLU(), nn.Linear(16, 16), nn.ReLU(),
                         nn.Linear(16, 4))


def test_refuses_partitions_with_random_ops():
    model = nn.Sequential(nn.Linear(4, 4), nn.Dropout(0.1), nn.Linear(4, 2))
    stage = PipelineStage(model, [3], chunks=2)
    with pytest.raises(ValueError, match='random numbers'):
        StepGraph(stage, F.mse_loss)
    ours = nn.Sequential(nn.Conv2d(3, 4, 1), Dropout2d(0.2))
    assert rng_modules(ours) == ['1']
    # p = 0 draws nothing
    assert rng_modules(nn.Sequential(nn.Dropout(0.0))) == []


def test_needs_a_warmup_step():
    stage = PipelineStage(_mlp(), [5], chunks=2)
    with pytest.raises(ValueError, match='warm-up'):
        StepGraph(stage, F.mse_loss, warmup=0)


def test_philox_pair_refuses_to_draw_inside_a_capture(monkeypatch):
    monkeypatch.setattr(torch.cuda, 'is_current_stream_capturing', lambda: True)
    with pytest.raises(RuntimeError, match='hipGraph capture'):
        rng.philox_pair(torch.device('cuda', 0), 16)


def test_cpu_steps_match_eager_training():
    a, b = _mlp(), _mlp()
    sa = PipelineStage(a, [5], chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [5], chunks=4, checkpoint='except_last')
    oa = torch.optim.SGD(sa.parameters(), lr=0.1)
    ob = torch.optim.SGD(sb.parameters(), lr=0.1)
    graph = StepGraph(sb, F.mse_loss, ob, warmup=1)
    torch.manual_seed(1)
    for _ in range(4):
        x, y = torch.randn(16, 8), torch.randn(16, 4)
        la = sa.train_step(x, y, F.mse_loss)
        oa.step()
        oa.zero_grad(set_to_none=True)
        lb = graph.step(x, y)
        assert torch.equal(la, lb)
    for pa, pb in zip(a.parameters(), b.parameters()):
        assert torch.equal(pa, pb)
    assert not graph.captured  # nothing to capture on a CPU stage


@pytest.mark.gpu
def test_graph_replays_match_eager_steps_on_gpu():
    """Tiny AmoebaNet-D (fused ReLU-Conv-BN ops, pools, BatchNorm running statistics,
    checkpoint recomputation): eager steps vs warm-up + capture + replays, with a new
    input every step (copied into the static buffers)."""
    from torchgpipe_amd.models import amoebanetd
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last')
    oa = torch.optim.SGD(sa.parameters(), lr=0.05)
    ob = torch.optim.SGD(sb.parameters(), lr=0.05)
    graph = StepGraph(sb, F.cross_entropy, ob, warmup=2)
    gen = torch.Generator(device=dev).manual_seed(3)
    for k in range(6):
        x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
        y = torch.randint(10, (8,), device=dev, generator=gen)
        la = sa.train_step(x, y, F.cross_entropy)
        oa.step()
        oa.zero_grad(set_to_none=True)
        lb = graph.step(x, y)
        torch.cuda.synchronize()
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6, msg=f'loss of step {k}')
    assert graph.captured
    for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pb, pa, rtol=1e-4, atol=1e-5, msg=name)
    for (name, ba), bb in zip(a.named_buffers(), b.buffers()):
        torch.testing.assert_close(bb, ba, rtol=1e-4, atol=1e-5, msg=name)


@pytest.mark.gpu
@pytest.mark.parametrize('graphed', [False, True])
def test_two_stream_cells_match_one_stream(graphed):
    """AmoebaNet cells with their independent nodes on two HIP streams (eager, and captured
    into a hipGraph) compute the one-stream model's losses, parameter gradients (which the
    fused ops on the side stream write themselves) and BatchNorm buffers, step after step.

    Gradients are compared per step (no optimizer: the update would amplify the
    legitimate fp32 differences of autograd summing a node's gradient contributions from
    the two streams in another order)."""
    from torchgpipe_amd.models import amoebanetd
    from torchgpipe_amd.models.amoebanet import set_cell_streams
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    set_cell_streams(b, True)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last')
    graph = StepGraph(sb, F.cross_entropy, None, warmup=2) if graphed else None
    gen = torch.Generator(device=dev).manual_seed(5)
    for k in range(5):
        x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
        y = torch.randint(10, (8,), device=dev, generator=gen)
        for p in sa.parameters():
            p.grad = None
        la = sa.train_step(x, y, F.cross_entropy)
        if graph is not None:
            lb = graph.step(x, y)
        else:
            for p in sb.parameters():
                p.grad = None
            lb = sb.train_step(x, y, F.cross_entropy)
        torch.cuda.synchronize()
        assert lb is not None and la is not None
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
            assert pb.grad is not None, name
            scale = pa.grad.abs().max().item() + 1e-12
            torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-4, atol=1e-5 * scale)
    for (name, ba), bb in zip(a.named_buffers(), b.buffers()):
        torch.testing.assert_close(bb, ba, rtol=1e-4, atol=1e-5)


def test_big_stack_worker_runs_calls_and_reraises():
    import threading
    from torchgpipe_amd.utils.bigstack import call_with_big_stack
    names = []
    assert call_with_big_stack(lambda: names.append(threading.current_thread().name) or 7) == 7
    assert names == ['tgpipe-big-stack']

    def deep(n):  # ~100 k Python frames would not fit the default thread stack
        return 0 if n == 0 else 1 + deep(n - 1)

    import sys
    limit = sys.getrecursionlimit()
    sys.setrecursionlimit(60000)
    try:
        assert call_with_big_stack(lambda: deep(50000)) == 50000
    finally:
        sys.setrecursionlimit(limit)
    with pytest.raises(ZeroDivisionError):
        call_with_big_stack(lambda: 1 / 0)


def test_big_stack_worker_keeps_the_callers_autograd_state():
    """Grad mode, inference mode and autocast follow the call to the worker thread, and a
    call made from the worker itself runs in place instead of deadlocking."""
    from torchgpipe_amd.utils.bigstack import call_with_big_stack

    def state():
        return (torch.is_grad_enabled(), torch.is_inference_mode_enabled(),
                torch.is_autocast_enabled('cpu'), torch.get_autocast_dtype('cpu'))

    assert call_with_big_stack(state)[:3] == (True, False, False)
    with torch.no_grad():
        assert call_with_big_stack(state)[0] is False
    with torch.inference_mode():
        assert call_with_big_stack(state)[1] is True
    with torch.autocast('cpu', dtype=torch.bfloat16):
        got = call_with_big_stack(state)
        assert got[2] is True and got[3] == torch.bfloat16
    assert call_with_big_stack(lambda: call_with_big_stack(lambda: 5)) == 5


@pytest.mark.gpu
def test_deep_two_stream_graph_replays_from_the_big_stack_thread():
    """A captured graph of ~40 k kernels forked and joined across two streams (the shape
    of the full AmoebaNet two-stream step that crashed hipGraphLaunch on the main thread,
    profiles/r3/capture_crash.md) replays from the big-stack worker with the exact
    result of its eager twin."""
    from torchgpipe_amd.utils.bigstack import call_with_big_stack
    dev = torch.device('cuda', 0)
    x = torch.zeros(64, device=dev)
    side = torch.cuda.Stream(dev)
    graph = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()

    def capture():
        with torch.cuda.graph(graph):
            main = torch.cuda.current_stream()
            for i in range(10000):
                side.wait_stream(main)
                with torch.cuda.stream(side):
                    x.add_(1.0)
                main.wait_stream(side)
                x.mul_(1.0)
                x.add_(1.0)

    capture()
    x.zero_()
    for _ in range(2):
        call_with_big_stack(graph.replay)
    torch.cuda.synchronize()
    assert torch.all(x == 40000.0)
