"""Which aten ops launch the non-native kernels of a pipeline partition: one micro-batch's
forward + backward of ResNet-101's / AmoebaNet-D(18,256)'s layers [lo, hi) under
``torch.profiler``, CPU ops with their CUDA kernel counts, grouped by a short Python stack.

    python benchmarks/diag/op_census.py --lo 260 --hi 370 --batch 22
    python benchmarks/diag/op_census.py --model amoebanet --lo 9 --hi 24 --batch 40
"""
import argparse
import os
import sys
from collections import Counter

import torch
import torch.nn.functional as F
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import amoebanetd, resnet101  # noqa: E402
from torchgpipe_amd.ops.fusion import relink  # noqa: E402
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--lo', type=int, default=260)
    p.add_argument('--hi', type=int, default=370)
    p.add_argument('--batch', type=int, default=22)
    p.add_argument('--model', choices=['resnet101', 'amoebanet'], default='resnet101')
    a = p.parse_args()
    dev = torch.device('cuda')
    if a.model == 'amoebanet':
        model = amoebanetd(num_classes=1000, num_layers=18, num_filters=256).to(dev)
    else:
        model = resnet101(num_classes=1000).to(dev)
    layers = list(model.children())
    head = torch.nn.Sequential(*layers[:a.lo])
    part = torch.nn.Sequential(*layers[a.lo:a.hi])
    relink(head)
    relink(part)
    image = torch.randn(a.batch, 3, 224, 224, device=dev)
    last = a.hi >= len(layers)
    target = torch.randint(0, 1000, (a.batch,), device=dev)

    def step():
        # one skip tracker for both: a residual stashed in the head pops in the partition
        with use_skip_tracker(SkipTracker()):
            with torch.no_grad():
                x = head(image)
            if isinstance(x, tuple):  # AmoebaNet's (x, skip) boundary
                y = part(tuple(t.detach().requires_grad_(True) for t in x))
            else:
                y = part(x.detach().requires_grad_(a.lo > 0))
            if last:
                F.cross_entropy(y, target).backward()
            else:
                y.backward(torch.ones_like(y))

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                 with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    # kernels per launching aten op (the op's own kernels, not its children's)
    kern = Counter()
    for e in prof.events():
        if e.device_type.name == 'CPU' and e.name.startswith('aten::'):
            names = [k.name for k in e.kernels]
            for n in names:
                if not n.startswith('void tgpipe') and 'tgpipe::' not in n:
                    stack = [s for s in (e.stack or [])
                             if 'torchgpipe_amd' in s or 'op_census' in s]
                    where = ' < '.join(s.split('/')[-1] for s in stack[:3])
                    kern[(e.name, n[:60], where)] += 1
    for (op, k, st), c in kern.most_common(40):
        print(f'{c:5d}  {op:32s} {k:60s} {st}')


if __name__ == '__main__':
    main()
