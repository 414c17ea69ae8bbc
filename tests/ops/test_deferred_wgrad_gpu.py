"""Deferred split weight gradients (ops/gradacc.py deferred_wgrad, csrc/conv_gemm.hip
launch_conv_gemm_wgrad_slab / slab_flush_kernel) against fp64 references and against the
per-micro-batch reduction they replace."""
import copy

import pytest
import torch
import torch.nn.functional as F

from torchgpipe_amd.ops import _ext, gradacc

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip('needs a GPU')
    assert _ext.available(), _ext.load_error()


def ops():
    return torch.ops.tgpipe


def rel_err(a, b):
    return ((a.double() - b.double()).norm() / (b.double().norm() + 1e-30)).item()


@pytest.mark.parametrize('geo_case', [
    ((8, 64, 28, 28), (96, 64, 1, 1), [1, 1, 1, 1, 0, 0, 0, 0]),
    ((4, 32, 28, 28), (48, 32, 1, 7), [1, 7, 1, 1, 0, 3, 0, 0]),
], ids=['1x1', '1x7'])
@pytest.mark.parametrize('splits', [(4, 4), (8, 2)], ids=['same-splits', 'changed-splits'])
def test_slab_accumulates_micro_batches_then_flushes(geo_case, splits):
    """Three micro-batches into one slab (the third with a different split count takes the
    reduce-into-slice-0 fallback when the counts differ), one flush into an existing
    gradient: equals grad + the fp64 sum of the three weight gradients."""
    xs, ws, geo = geo_case
    torch.manual_seed(0)
    wt = torch.randn(*ws, device='cuda') / (ws[1] * ws[2] * ws[3]) ** 0.5
    want = torch.zeros(ws, dtype=torch.float64, device='cuda')
    slab = torch.empty(0, device='cuda')
    try:
        for k in range(3):
            ops().conv_gemm_force_cfg(0, splits[0] if k < 2 else splits[1])
            x = torch.randn(*xs, device='cuda')
            z = ops().conv_gemm_forward(x, wt, geo, True)
            dz = torch.randn_like(z)
            x64 = x.double().requires_grad_(True)
            w64 = wt.double().requires_grad_(True)
            ref = F.conv2d(F.relu(x64), w64, padding=(geo[4], geo[5]))
            ref.backward(dz.double())
            want += w64.grad
            out = ops().conv_gemm_backward_weight(dz, x, wt, geo, True, None, slab, k == 0)
            assert out.data_ptr() == slab.data_ptr(), 'the split plan must defer into the slab'
    finally:
        ops().conv_gemm_force_cfg(-1)
    assert slab.numel() % wt.numel() == 0 and slab.numel() > wt.numel()
    grad = torch.randn_like(wt)
    want += grad.double()
    ops().wgrad_slab_flush([slab], [grad], [1])
    assert rel_err(grad, want) < 5e-6


def test_unsplit_plan_writes_the_gradient_directly():
    torch.manual_seed(0)
    x = torch.randn(2, 32, 8, 8, device='cuda')
    wt = torch.randn(32, 32, 1, 1, device='cuda')
    geo = [1, 1, 1, 1, 0, 0, 0, 0]
    dz = torch.randn(2, 32, 8, 8, device='cuda')
    slab = torch.empty(0, device='cuda')
    ops().conv_gemm_force_cfg(0, 1)
    try:
        out = ops().conv_gemm_backward_weight(dz, x, wt, geo, True, None, slab, True)
    finally:
        ops().conv_gemm_force_cfg(-1)
    assert slab.numel() == 0 and out.data_ptr() != slab.data_ptr()
    want = torch.einsum('nohw,nihw->oi', dz.double(), F.relu(x).double())
    assert rel_err(out.view(32, 32), want) < 5e-6


def test_flush_table_spans_several_launches():
    """More parameters than one flush launch's table, odd sizes (scalar tail path), fresh
    and accumulated gradients."""
    torch.manual_seed(0)
    slabs, grads, acc, want = [], [], [], []
    for k in range(53):
        numel = 1000 + 37 * k if k % 2 else 1024 * (k + 1)
        splits = 1 + k % 5
        s = torch.randn(splits * numel, device='cuda')
        g = torch.randn(numel, device='cuda')
        a = k % 3 != 0
        want.append(s.double().view(splits, numel).sum(0) + (g.double() if a else 0))
        slabs.append(s)
        grads.append(g)
        acc.append(int(a))
    ops().wgrad_slab_flush(slabs, grads, acc)
    for g, w in zip(grads, want):
        assert rel_err(g, w) < 1e-6


@pytest.mark.parametrize('cell_streams', [False, True])
def test_pipeline_stage_gradients_match_without_deferral(cell_streams, monkeypatch):
    """Tiny AmoebaNet-D through PipelineStage (4 micro-batches, checkpointing): gradients
    with the deferred slabs equal those of the per-micro-batch reduction, step after step
    (gradient accumulation across steps included)."""
    from torchgpipe_amd.models import amoebanetd
    from torchgpipe_amd.models.amoebanet import set_cell_streams
    from torchgpipe_amd.parallel import PipelineStage
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    if cell_streams:
        set_cell_streams(a, True)
        set_cell_streams(b, True)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last')
    gen = torch.Generator(device=dev).manual_seed(5)
    deferred_seen = 0
    for k in range(3):
        x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
        y = torch.randint(10, (8,), device=dev, generator=gen)
        if k != 1:  # step 1 accumulates onto step 0's gradients
            for p in list(sa.parameters()) + list(sb.parameters()):
                p.grad = None
        monkeypatch.setattr(gradacc, '_DEFER_ENABLED', False)
        la = sa.train_step(x, y, F.cross_entropy)
        monkeypatch.setattr(gradacc, '_DEFER_ENABLED', True)
        lb = sb.train_step(x, y, F.cross_entropy)
        torch.cuda.synchronize()
        deferred_seen = max(deferred_seen, sum(
            getattr(p, gradacc._SLAB_ATTR, [torch.empty(0)])[0].numel() > 0
            for p in sb.parameters()))
        torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
        for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
            assert pb.grad is not None, name
            scale = pa.grad.abs().max().item() + 1e-12
            torch.testing.assert_close(pb.grad, pa.grad, rtol=1e-4, atol=1e-5 * scale,
                                       msg=f'{name} step {k}')
    assert deferred_seen > 0, 'no weight gradient took the deferred path'
