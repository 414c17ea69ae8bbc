"""Memory benchmark: largest trainable U-Net / AmoebaNet per pipeline configuration.

Reference: ``benchmarks/unet-memory/main.py:22-78`` and
``benchmarks/amoebanetd-memory/main.py:22-73`` — train 2 steps, report
Σ over devices of peak reserved memory and the parameter count.

Multi-GPU configurations are measured **one stage at a time on one GPU**:
every stage of a multi-process pipeline owns one GPU and exactly the work of
:class:`~torchgpipe_amd.parallel.PipelineStage` (its layers, ``m`` checkpointed
micro-batch inputs + cross-stage skip tensors, its gradients and optimizer
state), so the per-stage peak measured here is that rank's peak.  The model is
built on the ``meta`` device; stage inputs and skip tensors get their shapes
from a meta-device forward of the preceding layers, and only the measured
stage is materialised on the GPU.

    python benchmarks/memory.py unet --experiment pipeline-8          # U-Net(48,160), 15.8 B
    python benchmarks/memory.py unet -B 11 -C 128 --balance 505 --chunks 32
"""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.checkpoint import Checkpointing  # noqa: E402
from torchgpipe_amd.microbatch import Batch  # noqa: E402
from torchgpipe_amd.models import amoebanetd, unet  # noqa: E402
from torchgpipe_amd.ops import conv as wino  # noqa: E402
from torchgpipe_amd.ops import gradacc  # noqa: E402
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker  # noqa: E402
from torchgpipe_amd.utils.meta import materialize  # noqa: E402

# (depth, channels) = U-Net (B = convs per cell, C = base channels) / AmoebaNet (L, D).
UNET_TABLE = {  # reference: benchmarks/unet-memory/main.py (input 32x3x192x192, SGD)
    'baseline': dict(depth=6, channels=72, balance=None, chunks=1),
    'pipeline-1': dict(depth=11, channels=128, balance=[505], chunks=32),
    'pipeline-2': dict(depth=24, channels=128, balance=[526, 551], chunks=32),
    'pipeline-4': dict(depth=24, channels=160, balance=[472, 54, 36, 515], chunks=32),
    'pipeline-8': dict(depth=48, channels=160, balance=[800, 140, 62, 36, 36, 36, 36, 987],
                       chunks=128),
}
AMOEBA_TABLE = {  # reference: benchmarks/amoebanetd-memory/main.py (128x3x224x224, RMSprop)
    'baseline': dict(depth=18, channels=208, balance=None, chunks=1),
    'pipeline-1': dict(depth=18, channels=416, balance=[24], chunks=128),
    'pipeline-2': dict(depth=18, channels=544, balance=[16, 8], chunks=128),
    'pipeline-4': dict(depth=36, channels=544, balance=[16, 12, 7, 7], chunks=128),
    'pipeline-8': dict(depth=72, channels=512, balance=[23, 16, 11, 6, 6, 5, 5, 6], chunks=128),
}


# transform-cache budget of the measured stages: a fraction of their uncached first-step peak
CACHE_FRACTION = float(os.environ.get('TGPIPE_WINOGRAD_CACHE_FRACTION', '0.15'))


def build(kind: str, b: int, c: int) -> nn.Sequential:
    """U-Net(B, C) = unet(depth=5, num_convs=B, base_channels=C); AmoebaNet-D(L, D)."""
    with torch.device('meta'):
        if kind == 'unet':
            return unet(depth=5, num_convs=b, base_channels=c, input_channels=3,
                        output_channels=1)
        return amoebanetd(num_classes=1000, num_layers=b, num_filters=c)


def stage_inputs(layers, lo, mb, shape):  # type: ignore[no-untyped-def]
    """Shapes of stage ``lo``'s input and of the skips alive at its start (meta forward)."""
    tracker = SkipTracker()
    with torch.no_grad(), use_skip_tracker(tracker):
        batch = Batch(torch.empty(mb, *shape, device='meta'))
        for layer in layers[:lo]:
            layer.eval()
            batch = batch.call(layer)
    return batch, dict(tracker.tensors)


def measure_stage(kind, layers, lo, hi, batch_size, chunks, shape, checkpoint, device):  # type: ignore[no-untyped-def]
    mb = max(1, batch_size // chunks)
    m = len(torch.empty(batch_size).chunk(chunks))
    meta_in, meta_skips = stage_inputs(layers, lo, mb, shape)
    part = nn.Sequential(*layers[lo:hi])
    materialize(part, device)
    part.train()
    params = sum(p.numel() for p in part.parameters())
    if kind == 'unet':
        opt = torch.optim.SGD(part.parameters(), lr=0.1)
    else:
        opt = torch.optim.RMSprop(part.parameters(), lr=0.1)

    def real(t):  # type: ignore[no-untyped-def]
        return torch.rand(t.shape, device=device) if t is not None else None

    stop = {'always': m, 'except_last': m - 1, 'never': 0}[checkpoint]
    last = hi == len(layers)
    torch.cuda.reset_peak_memory_stats(device)
    # as PipelineStage does: the first step runs without cached weight transforms, and its
    # peak sizes the cache for the second (ops/conv.py size_cache_budget) -- here in the
    # memory-lean mode, at most CACHE_FRACTION of that peak
    wino.hold_cache(device)
    cache_budget = 0
    for step in range(2):
        wino.new_step()
        if step == 1:
            cache_budget = wino.size_cache_budget(device, torch.cuda.max_memory_allocated(device),
                                                  CACHE_FRACTION)
        cells = []
        for i in range(m):
            acts = [real(t).requires_grad_(lo > 0) for t in meta_in]
            skips = {k: real(v) for k, v in meta_skips.items()}

            def fn(flat, skips=skips):  # type: ignore[no-untyped-def]
                tr = SkipTracker()
                tr.tensors = dict(skips)
                with use_skip_tracker(tr):
                    out = part(flat[0] if meta_in.atomic else tuple(flat))
                return tuple(Batch(out))

            if i < stop:
                chk = Checkpointing(fn, Batch(tuple(acts)))
                out = list(chk.checkpoint())
            else:
                chk, out = None, list(fn(tuple(acts)))
            cells.append((chk, out))
        # as PipelineStage.backward: split weight gradients deferred into per-parameter
        # slabs, flushed once after the last micro-batch (ops/gradacc.py)
        scope = gradacc.deferred_wgrad(device)
        scope.__enter__()
        for k in reversed(range(len(cells))):
            chk, out = cells[k]
            if chk is not None:
                # as PipelineStage(direct_backward=True): recompute, then back-propagate
                # through the recomputed graph (the Checkpoint node never runs)
                chk.recompute_now()
                out, _ = chk.take_recomputed()
            cells[k] = (None, [])
            ys = [y for y in out if y.requires_grad]
            if last and kind == 'unet':
                loss = F.binary_cross_entropy_with_logits(ys[0], torch.ones_like(ys[0]))
                loss.backward()
            elif last:
                loss = F.cross_entropy(ys[0], torch.zeros(ys[0].size(0), dtype=torch.long,
                                                          device=device))
                loss.backward()
            else:
                torch.autograd.backward(ys, [torch.ones_like(y) for y in ys])
        scope.__exit__(None, None, None)
        del cells
        opt.step()
        if step == 1:  # the model state at its largest: parameters, gradients, optimizer
            grad_bytes = sum(q.grad.numel() * q.grad.element_size() for q in part.parameters()
                             if q.grad is not None)
            opt_bytes = sum(t.numel() * t.element_size() for st in opt.state.values()
                            for t in st.values() if torch.is_tensor(t) and t.is_cuda)
            slab_bytes = 0
            for q in part.parameters():
                entry = getattr(q, '_tgpipe_wgrad_slab', None)  # [slab, step]
                if entry and torch.is_tensor(entry[0]):
                    slab_bytes += entry[0].numel() * entry[0].element_size()
        opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize(device)
    peak = torch.cuda.max_memory_reserved(device)
    peak_alloc = torch.cuda.max_memory_allocated(device)
    cached = wino.cache_bytes()
    param_bytes = sum(q.numel() * q.element_size() for q in part.parameters())
    # what the peak is made of: the reference reports model memory (parameters + gradients +
    # optimizer state) and peak activation memory (benchmarks/amoebanetd-memory/README.md)
    parts = {'param_gib': param_bytes, 'grad_gib': grad_bytes, 'optimizer_state_gib': opt_bytes,
             'transform_cache_gib': cached, 'wgrad_slab_gib': slab_bytes,
             'activations_and_workspace_gib': max(0, peak_alloc - param_bytes - grad_bytes
                                                  - opt_bytes - cached - slab_bytes),
             'allocator_reserve_gib': max(0, peak - peak_alloc)}
    parts = {k: round(v / 2 ** 30, 3) for k, v in parts.items()}
    del opt
    wino.clear_winograd_caches(part)
    part.to_empty(device='meta')  # release this stage before measuring the next one
    del part
    torch.cuda.empty_cache()
    return params, peak, cache_budget, cached, parts


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    p.add_argument('model', choices=['unet', 'amoebanet'])
    p.add_argument('--experiment', default=None, help='reference table row, e.g. pipeline-8')
    p.add_argument('--depth', '-B', type=int, default=None,
                   help='U-Net B (convs per cell) or AmoebaNet L (layers)')
    p.add_argument('--channels', '-C', type=int, default=None,
                   help='U-Net C (base channels) or AmoebaNet D (filters)')
    p.add_argument('--balance', nargs='*', default=None,
                   help="layers per stage, or 'params N' to split N ways by parameter bytes")
    p.add_argument('--chunks', type=int, default=None)
    p.add_argument('--batch', type=int, default=None)
    p.add_argument('--stages', type=int, nargs='*', default=None)
    p.add_argument('--checkpoint', default='except_last')
    p.add_argument('--out', default=None)
    args = p.parse_args()

    table = UNET_TABLE if args.model == 'unet' else AMOEBA_TABLE
    cfg = dict(table[args.experiment]) if args.experiment else {}
    depth = args.depth or cfg['depth']
    channels = args.channels or cfg['channels']
    chunks = args.chunks or cfg.get('chunks', 1)
    batch = args.batch or (32 if args.model == 'unet' else 128)
    shape = (3, 192, 192) if args.model == 'unet' else (3, 224, 224)
    model = build(args.model, depth, channels)
    layers = list(model)
    if args.balance and args.balance[0] == 'params':
        from torchgpipe_amd.balance.blockpartition import solve_splits
        cost = [sum(p.numel() for p in layer.parameters()) + 1 for layer in layers]
        balance = solve_splits(cost, int(args.balance[1]))
    elif args.balance:
        balance = [int(v) for v in args.balance]
    else:
        balance = cfg.get('balance') or [len(layers)]
    assert sum(balance) == len(layers), (sum(balance), len(layers))
    total_params = sum(p.numel() for p in model.parameters())
    device = torch.device('cuda', 0)

    bounds = [0]
    for b in balance:
        bounds.append(bounds[-1] + b)
    stages = args.stages if args.stages is not None else list(range(len(balance)))
    rows = []
    t0 = time.time()
    for k in stages:
        params, peak, budget, cached, parts = measure_stage(
            args.model, layers, bounds[k], bounds[k + 1], batch, chunks, shape,
            args.checkpoint, device)
        row = {'stage': k, 'layers': [bounds[k], bounds[k + 1]], 'params': params,
               'peak_reserved_gib': round(peak / 2 ** 30, 2),
               'transform_cache_budget_gib': round(budget / 2 ** 30, 2),
               'transform_cache_gib': round(cached / 2 ** 30, 2), 'breakdown': parts}
        rows.append(row)
        print(json.dumps(row), f'({time.time() - t0:.0f}s)', flush=True)
    summary = {'model': args.model, 'depth': depth, 'channels': channels, 'balance': balance,
               'chunks': chunks, 'batch': batch, 'total_params': total_params,
               'total_params_billion': round(total_params / 1e9, 3),
               'sum_peak_reserved_gib': round(sum(r['peak_reserved_gib'] for r in rows), 2),
               'max_stage_peak_gib': max(r['peak_reserved_gib'] for r in rows),
               'sum_breakdown_gib': {key: round(sum(r['breakdown'][key] for r in rows), 2)
                                     for key in rows[0]['breakdown']},
               'device': torch.cuda.get_device_name(device),
               'device_total_gib': round(torch.cuda.get_device_properties(device).total_memory
                                         / 2 ** 30, 1),
               'stages': rows}
    print(json.dumps({k: v for k, v in summary.items() if k != 'stages'}), flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            json.dump(summary, f, indent=1)


if __name__ == '__main__':
    main()
