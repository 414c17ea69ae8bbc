"""Host (CPU) cost of AmoebaNet cells and ResNet-101 blocks at launch-bound sizes.

The AmoebaNet m32 and ResNet p4 / p8 pipeline stages are launch-bound: the stage harness
reports host enqueue at 0.95-1.0 of the step (``profiles/r5/harness/``), and
``torch.profiler`` puts most of it in Python around the fused ops
(``profiles/r5/host_profile.md``).  This times one cell / block forward (with grad) and
forward + backward on inputs too small to keep the GPU busy, so the wall time per call is
the host's enqueue cost.

    python benchmarks/host_cell.py --out gpurun_out/host_cell.json
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchgpipe_amd.ops import _ext  # noqa: E402


def host_us(fn, iters):  # type: ignore[no-untyped-def]
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    host = (time.perf_counter() - t) / iters * 1e6
    torch.cuda.synchronize()
    return round(host, 1)


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--iters', type=int, default=200)
    p.add_argument('--out', default=None)
    a = p.parse_args()
    _ext.require()
    dev = torch.device('cuda')
    rows = {}

    # stream / event primitives the multi-stream cells use per node
    side = torch.cuda.Stream(dev)
    main = torch.cuda.current_stream(dev)
    t = torch.randn(16, device=dev)
    ev = torch.cuda.Event()

    def ctx():  # type: ignore[no-untyped-def]
        with torch.cuda.stream(side):
            pass

    def setstream():  # type: ignore[no-untyped-def]
        torch.cuda.set_stream(side)
        torch.cuda.set_stream(main)

    rows['stream_context_us'] = host_us(ctx, 2000)
    rows['set_stream_pair_us'] = host_us(setstream, 2000)
    rows['event_new_record_us'] = host_us(lambda: torch.cuda.Event().record(side), 2000)
    rows['event_record_us'] = host_us(lambda: ev.record(side), 2000)
    rows['wait_event_us'] = host_us(lambda: main.wait_event(ev), 2000)
    rows['record_stream_us'] = host_us(lambda: t.record_stream(side), 2000)
    rows['current_stream_us'] = host_us(lambda: torch.cuda.current_stream(dev), 2000)

    from torchgpipe_amd.models.amoebanet import amoebanetd, set_cell_streams
    model = amoebanetd(num_classes=10, num_layers=6, num_filters=32).to(dev).train()
    layers = list(model)
    cell = layers[3]  # a normal cell
    x = torch.randn(2, 3, 224, 224, device=dev)
    with torch.no_grad():
        h = x
        for layer in layers[:3]:
            h = layer(h)
    s = tuple(t.detach().requires_grad_(True) for t in h) if isinstance(h, tuple) else \
        h.detach().requires_grad_(True)
    for streams in (0, 3):
        set_cell_streams(cell, streams)

        def fwd():  # type: ignore[no-untyped-def]
            return cell(s)

        def fwd_bwd():  # type: ignore[no-untyped-def]
            out, _ = cell(s)
            out.sum().backward()

        rows[f'amoeba_cell_fwd_streams{streams}'] = host_us(fwd, a.iters)
        rows[f'amoeba_cell_fwd_bwd_streams{streams}'] = host_us(fwd_bwd, a.iters)

    from torchgpipe_amd.models.resnet import resnet101
    from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker
    net = resnet101(num_classes=1000).to(dev).train()
    seq = list(net)
    # one whole bottleneck of layer3 (11 flattened layers: identity stash ... relu3; stem 4 +
    # layer1 33 + layer2 44 layers before layer3), 14^2 x 1024 at 2 images
    start = 4 + 33 + 44 + 11 * 5
    block = seq[start:start + 11]
    with torch.no_grad(), use_skip_tracker(SkipTracker()):
        h = torch.randn(2, 3, 224, 224, device=dev)
        for layer in seq[:start]:
            h = layer(h)
    hb = h.detach().requires_grad_(True)

    def rfwd():  # type: ignore[no-untyped-def]
        with use_skip_tracker(SkipTracker()):
            y = hb
            for layer in block:
                y = layer(y)
        return y

    def rfwd_bwd():  # type: ignore[no-untyped-def]
        rfwd().sum().backward()

    rows['resnet_bottleneck_fwd'] = host_us(rfwd, a.iters)
    rows['resnet_bottleneck_fwd_bwd'] = host_us(rfwd_bwd, a.iters)
    print(json.dumps(rows))
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
