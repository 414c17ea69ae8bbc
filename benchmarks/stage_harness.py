"""Run ONE pipeline stage of a multi-GPU U-Net / AmoebaNet / ResNet-101 experiment on one GPU.

The stage is the real engine -- :class:`~torchgpipe_amd.parallel.PipelineStage` as rank
``k`` of ``len(balance)`` -- on a loopback transport
(:class:`~torchgpipe_amd.parallel.loopback.LoopbackP2P`): its receives return, at once,
the boundary activations and skips the preceding stages produce (computed here by running
the model's prefix on one micro-batch) or random output gradients, and its sends are
dropped.  Every step is what the rank does on a multi-GPU node (``m`` forwards, ``m``
recomputations and backwards on the lanes, multi-stream cells, captured cells with
``--graph-cells``, the SGD update) minus the waits on its neighbours, so

* ``device_ms`` is the stage's compute per step (GPU busy span, events on the main stream),
* ``host_ms`` the host's enqueue time per step (Python, autograd, dispatcher, launches),
* ``host_share`` = host / device: above 1 the stage is launch-bound; the pipeline needs it
  well below 1 so that host hiccups stay off the critical path.

The slowest stage's ``device_ms`` bounds the pipeline's step time (plus the fill/drain
bubble, ``torchgpipe_amd.balance.simulate``).

    python benchmarks/stage_harness.py --model amoebanet --balance 2 2 2 3 3 4 4 4 \\
        --chunks 32 --batch 1280 --graph-cells
"""
import argparse
import json
import os
import sys
import time
from typing import Dict, List

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.microbatch import Batch  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402
from torchgpipe_amd.parallel.loopback import LoopbackP2P  # noqa: E402
from torchgpipe_amd.parallel.stage import signature_of  # noqa: E402
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker  # noqa: E402

SHAPES = {'unet': (3, 192, 192), 'amoebanet': (3, 224, 224), 'resnet101': (3, 224, 224)}


def build(kind: str, dev: torch.device) -> torch.nn.Sequential:
    from torchgpipe_amd.models import amoebanetd, resnet101, unet
    with dev:
        if kind == 'unet':
            return unet(depth=5, num_convs=5, base_channels=64)
        if kind == 'amoebanet':
            return amoebanetd(num_classes=1000, num_layers=18, num_filters=256)
        return resnet101(num_classes=1000)


def sent_bytes(transport: LoopbackP2P) -> Dict[str, int]:
    """``{'act->j' / 'skip->j': bytes}`` of micro-batch 0's sends."""
    out: Dict[str, int] = {}
    for (kind, i, dst), metas in transport._sent.items():
        if i != 0 or kind not in ('act', 'skip'):
            continue
        nbytes = 0
        for m in metas:
            numel = 1
            for d in m.shape:
                numel *= d
            nbytes += numel * torch.empty(0, dtype=m.dtype).element_size()
        out[f'{kind}->{dst}'] = out.get(f'{kind}->{dst}', 0) + nbytes
    return out


def run_stage(args: argparse.Namespace, k: int, dev: torch.device) -> Dict[str, object]:
    torch.manual_seed(0)
    model = build(args.model, dev).train()
    shape = SHAPES[args.model]
    layers = list(model)
    bounds = [0]
    for b in args.balance:
        bounds.append(bounds[-1] + b)
    lo, hi = bounds[k], bounds[k + 1]
    mb = -(-args.batch // args.chunks)

    # the boundary tensors of this stage: the prefix's output and the skips still in flight
    tracker = SkipTracker()
    with torch.no_grad(), use_skip_tracker(tracker):
        batch = Batch(torch.rand(mb, *shape, device=dev))
        for layer in layers[:lo]:
            batch = batch.call(layer)
    acts, atomic = [t.detach() for t in batch], batch.atomic
    pending = dict(tracker.tensors)
    del batch, tracker

    auto = args.model == 'unet' or (args.model == 'resnet101' and len(args.balance) == 1)
    lanes = {'auto': auto, 'on': True, 'off': False}[args.lanes]
    # placeholder transport until the stage knows its skip routes
    sizes = [len(c) for c in torch.empty(args.batch, 0).chunk(args.chunks)]
    transport = LoopbackP2P(dev, acts, atomic, {}, sizes)
    # (as bench.py: forward and recompute lanes for U-Net, and for ResNet-101 at pipeline-1
    # only; AmoebaNet runs its cells on several streams instead)
    recompute_lane = lanes
    stage = PipelineStage(model, args.balance, rank=k, device=dev, chunks=args.chunks,
                          checkpoint=args.checkpoint, transport=transport,
                          overlap_recompute=recompute_lane, overlap_forward=lanes,
                          graph_cells=args.graph_cells,
                          backward_thread=args.backward_thread)
    skips: Dict[int, List[torch.Tensor]] = {}
    for src, key in stage.in_skips:
        skips.setdefault(src, []).append(pending[key])
    transport.skips = skips
    del pending
    if args.cell_streams and args.model == 'amoebanet':
        from torchgpipe_amd.models.amoebanet import set_cell_streams
        set_cell_streams(stage.partition, args.cell_streams)

    x = torch.rand(args.batch, *shape, device=dev) if stage.is_first else None
    if args.model == 'unet':
        target = torch.ones(args.batch, 1, 192, 192, device=dev) if stage.is_last else None
        loss_fn = F.binary_cross_entropy_with_logits
    else:
        target = torch.randint(1000, (args.batch,), device=dev) if stage.is_last else None
        loss_fn = F.cross_entropy
    signature = signature_of(torch.empty(args.batch, *shape, device='meta'))
    optimizer = torch.optim.SGD(stage.parameters(), lr=0.1)

    def step() -> None:
        stage.train_step(x, target, loss_fn, signature=signature)
        optimizer.step()
        optimizer.zero_grad(set_to_none=True)

    t0 = time.perf_counter()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    warm_s = time.perf_counter() - t0

    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    seg = stage._segments
    launch0 = seg.launch_s if seg is not None else 0.0
    e0.record()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    host_ms = (time.perf_counter() - t0) * 1e3 / args.steps
    launch_ms = ((seg.launch_s - launch0) * 1e3 / args.steps) if seg is not None else None
    e1.record()
    e1.synchronize()
    wall_ms = (time.perf_counter() - t0) * 1e3 / args.steps
    dev_ms = e0.elapsed_time(e1) / args.steps
    idle_launch_ms = None
    if seg is not None and seg.cells and seg.cells[0].fwd is not None:
        # one forward graph launched on an idle GPU: the launch's own host cost
        torch.cuda.synchronize(dev)
        t1 = time.perf_counter()
        seg.cells[0].fwd.replay()
        idle_launch_ms = (time.perf_counter() - t1) * 1e3
        torch.cuda.synchronize(dev)
    if args.torch_profile:
        # one more step under torch.profiler (CPU activities of every thread, the autograd
        # engine's included): where the host time of a launch-bound stage goes
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU]) as prof:
            step()
            torch.cuda.synchronize(dev)
        with open(f'{args.torch_profile}_stage{k}.txt', 'w') as f:
            f.write(prof.key_averages().table(sort_by='self_cpu_time_total', row_limit=60,
                                              max_name_column_width=70))
    row = {'stage': k, 'layers': [lo, hi], 'graph_cells': args.graph_cells,
           'backward_thread': args.backward_thread,
           'graph_phase': stage.graph_phase, 'lanes': lanes,
           'host_ms': round(host_ms, 2), 'wall_ms': round(wall_ms, 2),
           'device_ms': round(dev_ms, 2), 'host_share': round(host_ms / dev_ms, 3),
           # captured cells: host time inside graph launches (enqueueing each graph's nodes,
           # and waiting whenever the GPU's queue is full) vs the rest (Python, transfers)
           'graph_launch_ms': None if launch_ms is None else round(launch_ms, 2),
           'host_outside_launch_share': None if launch_ms is None
           else round((host_ms - launch_ms) / dev_ms, 3),
           'idle_fwd_graph_launch_ms': None if idle_launch_ms is None
           else round(idle_launch_ms, 3),
           'warmup_s': round(warm_s, 1),
           'peak_mem_gib': round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
           # bytes this stage sends per micro-batch, per (kind, destination stage): the
           # boundary activation and the cross-stage skips (their gradients come back the
           # same size) -- the transfer model of scripts/r5/predict.py
           'sent_bytes': sent_bytes(transport)}
    del stage, optimizer, model, x, target, acts, skips, transport
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    return row


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__,
                                formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument('--model', choices=sorted(SHAPES), default='unet')
    p.add_argument('--balance', type=int, nargs='+', required=True)
    p.add_argument('--chunks', type=int, required=True)
    p.add_argument('--batch', type=int, required=True)
    p.add_argument('--stages', type=int, nargs='*', default=None)
    p.add_argument('--checkpoint', default='except_last')
    p.add_argument('--graph-cells', action='store_true',
                   help='captured cells (PipelineStage(graph_cells=True))')
    p.add_argument('--torch-profile', default=None,
                   help='path prefix: one extra step under torch.profiler, op table per stage')
    p.add_argument('--backward-thread', action='store_true',
                   help='backward issued from a helper thread (PipelineStage(backward_thread))')
    p.add_argument('--lanes', choices=['auto', 'on', 'off'], default='auto',
                   help='forward / recompute lanes (auto: on for U-Net, as bench.py)')
    p.add_argument('--cell-streams', type=int, default=3,
                   help='AmoebaNet: streams per cell (0: one stream; bench.py: 3)')
    p.add_argument('--warmup', type=int, default=3)
    p.add_argument('--steps', type=int, default=2)
    p.add_argument('--out', default=None)
    args = p.parse_args()
    if args.graph_cells and args.warmup < 4:
        args.warmup = 4  # two eager steps, the capture, a first replay
    dev = torch.device('cuda', 0)
    results = []
    for k in (args.stages if args.stages else range(len(args.balance))):
        row = run_stage(args, k, dev)
        results.append(row)
        print(json.dumps(row), flush=True)
    if args.out:
        with open(args.out, 'w') as f:
            json.dump({'args': vars(args), 'stages': results}, f, indent=1)


if __name__ == '__main__':
    main()
