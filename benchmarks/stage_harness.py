"""Run ONE pipeline stage of a multi-GPU U-Net/AmoebaNet experiment on one GPU.

Measures what a stage rank does per step — ``m`` checkpointed forwards, ``m``
recomputes and backwards — with real inputs/skips of the right shapes, and
reports device-busy time vs host wall time.  Host time ≫ device time means the
stage is launch-bound (a hipGraph candidate); device time per stage validates
the balance simulator (``torchgpipe_amd.balance.simulate``).

    python benchmarks/stage_harness.py --balance 18 27 29 23 25 33 44 42 --chunks 40 --batch 640
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.checkpoint import Checkpointing  # noqa: E402
from torchgpipe_amd.microbatch import Batch  # noqa: E402
from torchgpipe_amd.models import amoebanetd, unet  # noqa: E402
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--model', choices=['unet', 'amoebanet'], default='unet')
    p.add_argument('--balance', type=int, nargs='+', required=True)
    p.add_argument('--chunks', type=int, required=True)
    p.add_argument('--batch', type=int, required=True)
    p.add_argument('--stages', type=int, nargs='*', default=None)
    p.add_argument('--checkpoint', default='except_last')
    p.add_argument('--out', default=None)
    p.add_argument('--cell-streams', type=int, default=0,
                   help='AmoebaNet: streams per cell (0: one stream; bench.py uses 3 eager)')
    args = p.parse_args()

    dev = torch.device('cuda', 0)
    model = unet() if args.model == 'unet' else amoebanetd(1000, 18, 256)
    shape = (3, 192, 192) if args.model == 'unet' else (3, 224, 224)
    model.to(dev).train()
    if args.cell_streams and args.model == 'amoebanet':
        from torchgpipe_amd.models.amoebanet import set_cell_streams
        set_cell_streams(model, args.cell_streams)
    layers = list(model)
    mb = args.batch // args.chunks
    m = args.chunks
    stop = {'always': m, 'except_last': m - 1, 'never': 0}[args.checkpoint]

    bounds = [0]
    for b in args.balance:
        bounds.append(bounds[-1] + b)
    results = []
    stages = args.stages if args.stages else list(range(len(args.balance)))

    for k in stages:
        lo, hi = bounds[k], bounds[k + 1]
        # Produce this stage's input (and the skips stashed before it) once.
        tracker = SkipTracker()
        with torch.no_grad(), use_skip_tracker(tracker):
            x = torch.rand(mb, *shape, device=dev)
            batch = Batch(x)
            for layer in layers[:lo]:
                batch = batch.call(layer)
        saved_skips = dict(tracker.tensors)
        part = torch.nn.Sequential(*layers[lo:hi])
        inputs = [t.detach() for t in batch]
        atomic = batch.atomic

        def fn(flat, part=part):
            tr = SkipTracker()
            tr.tensors = dict(saved_skips)
            with use_skip_tracker(tr):
                out = part(flat[0] if atomic else tuple(flat))
            b = Batch(out)
            return tuple(b)

        def step():
            cells = []
            for i in range(m):
                leaves = [t.detach().requires_grad_(k > 0 and t.is_floating_point())
                          for t in inputs]
                if i < stop:
                    chk = Checkpointing(fn, Batch(tuple(leaves)))
                    out = list(chk.checkpoint())
                else:
                    chk = None
                    out = list(fn(tuple(leaves)))
                cells.append((chk, out))
            for chk, out in reversed(cells):
                if chk is not None:
                    chk.recompute_now()
                ys = [y for y in out if y.requires_grad]
                torch.autograd.backward(ys, [torch.ones_like(y) for y in ys])
            part.zero_grad(set_to_none=True)

        step()
        torch.cuda.synchronize()
        reps = 2
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        for _ in range(reps):
            step()
        host_ms = (time.perf_counter() - t0) * 1e3 / reps
        e1.record()
        e1.synchronize()
        wall_ms = (time.perf_counter() - t0) * 1e3 / reps
        dev_ms = e0.elapsed_time(e1) / reps
        row = {'stage': k, 'layers': [lo, hi], 'host_enqueue_ms': round(host_ms, 2),
               'wall_ms': round(wall_ms, 2), 'device_ms': round(dev_ms, 2),
               'per_cell_ms': round(wall_ms / m, 3)}
        results.append(row)
        print(json.dumps(row), flush=True)

    if args.out:
        with open(args.out, 'w') as f:
            json.dump({'args': vars(args), 'stages': results}, f, indent=1)


if __name__ == '__main__':
    main()
