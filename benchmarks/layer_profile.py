"""Per-layer forward / backward device time of a benchmark model (HIP events).

Feeds MI355X-specific balance tables: the reference's balances were tuned on
Tesla P40 + cuDNN; MIOpen on MI355X has a different cost profile per layer.

    python benchmarks/layer_profile.py --model unet --micro-batch 16 --out prof.json
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.microbatch import Batch  # noqa: E402
from torchgpipe_amd.models import amoebanetd, unet  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--model', choices=['unet', 'amoebanet'], default='unet')
    p.add_argument('--micro-batch', type=int, nargs='+', default=[16])
    p.add_argument('--iters', type=int, default=5)
    p.add_argument('--out', default='gpurun_out/layer_profile.json')
    args = p.parse_args()

    dev = torch.device('cuda', 0)
    if args.model == 'unet':
        model = unet().to(dev)
        shape = (3, 192, 192)
    else:
        model = amoebanetd(num_classes=1000, num_layers=18, num_filters=256).to(dev)
        shape = (3, 224, 224)
    model.train()
    names = [n for n, _ in model.named_children()]
    result = {'model': args.model, 'names': names, 'profiles': {}}

    for mb in args.micro_batch:
        fwd = [0.0] * len(model)
        bwd = [0.0] * len(model)
        out_bytes = [0] * len(model)
        t0 = time.time()
        for it in range(args.iters + 1):
            batch = Batch(torch.rand(mb, *shape, device=dev))
            from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker
            tracker = SkipTracker()
            with use_skip_tracker(tracker):
                for i, layer in enumerate(model):
                    inputs = tuple(x.detach().requires_grad_(x.is_floating_point())
                                   for x in batch)
                    b = Batch(inputs[0]) if batch.atomic else Batch(inputs)
                    e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                    e0.record()
                    out = b.call(layer)
                    e1.record()
                    grads = [torch.ones_like(y) for y in out if y.requires_grad]
                    ys = [y for y in out if y.requires_grad]
                    if ys:
                        torch.autograd.backward(ys, grads, retain_graph=False)
                    e2.record()
                    e2.synchronize()
                    if it > 0:
                        fwd[i] += e0.elapsed_time(e1) / args.iters
                        bwd[i] += e1.elapsed_time(e2) / args.iters
                    out_bytes[i] = sum(y.numel() * y.element_size() for y in out)
                    batch = Batch(tuple(y.detach() for y in out)) if not out.atomic \
                        else Batch(out.tensor.detach())
                    model.zero_grad(set_to_none=True)
            print(f'[layer_profile] mb={mb} iter {it} done at {time.time() - t0:.1f}s',
                  file=sys.stderr, flush=True)
        result['profiles'][str(mb)] = {'fwd_ms': fwd, 'bwd_ms': bwd, 'out_bytes': out_bytes,
                                       'total_fwd_ms': sum(fwd), 'total_bwd_ms': sum(bwd)}
        print(f'mb={mb}: fwd {sum(fwd):.2f} ms, bwd {sum(bwd):.2f} ms', flush=True)

    os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
    with open(args.out, 'w') as f:
        json.dump(result, f)


if __name__ == '__main__':
    main()
