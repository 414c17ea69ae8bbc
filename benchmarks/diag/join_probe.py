"""Does each ResNet-101 residual join run fused (ops/fusion.py pending_join) inside a
partition, and how many ReLU layers fall back to F.relu?  One micro-batch of layers [lo, hi)
under a plain skip tracker and under PipelineStage's portal tracker.

    python benchmarks/diag/join_probe.py --lo 260 --hi 370 --batch 22
"""
import argparse
import os
import sys
from collections import Counter

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import resnet101  # noqa: E402
from torchgpipe_amd.ops import fusion  # noqa: E402
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker  # noqa: E402

COUNT = Counter()
_join = fusion.pending_join
_add_relu = fusion.add_relu
_relu_fwd = fusion.ReLU.forward


def pending_join(x, join, identity):
    y = _join(x, join, identity)
    COUNT['join fused' if y is not None else 'join not fused'] += 1
    if y is None:
        COUNT['x has pending mark' if getattr(x, fusion._PENDING, None) else 'x lost mark'] += 1
    return y


def relu_forward(self, input):
    COUNT['ReLU passthrough' if getattr(input, fusion._DONE_RELU, False) else 'ReLU F.relu'] += 1
    return _relu_fwd(self, input)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--lo', type=int, default=260)
    p.add_argument('--hi', type=int, default=370)
    p.add_argument('--batch', type=int, default=22)
    a = p.parse_args()
    import torchgpipe_amd.models.resnet as rn
    rn.pending_join = pending_join
    fusion.ReLU.forward = relu_forward
    dev = torch.device('cuda')
    model = resnet101(num_classes=1000).to(dev)
    layers = list(model.children())
    head = torch.nn.Sequential(*layers[:a.lo])
    part = torch.nn.Sequential(*layers[a.lo:a.hi])
    fusion.relink(head)
    fusion.relink(part)
    image = torch.randn(a.batch, 3, 224, 224, device=dev)
    with use_skip_tracker(SkipTracker()):
        with torch.no_grad():
            x = head(image)
        COUNT.clear()
        y = part(x.detach().requires_grad_(True))
        y.float().sum().backward()
    print('plain tracker:', dict(COUNT))


if __name__ == '__main__':
    main()
