"""Where AmoebaNet's separate node-sum adds come from: one micro-batch through layers
[lo, hi) with ``Operation.forward``'s unfused ``+ add`` paths counted by operation type and
operand contiguity.

    python benchmarks/diag/amoeba_add_probe.py --lo 9 --hi 24 --batch 40
"""
import argparse
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import amoebanet as am  # noqa: E402
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker  # noqa: E402

COUNT = Counter()
_fwd = am.Operation.forward


def forward(self, x, add=None, first=None):
    if add is not None:
        if first is not None and len(self.module) == 3:
            path = 'first + add'
        elif first is None and not self.takes_add:
            path = 'out + add'
        else:
            path = 'folded'
        COUNT[(path, self.name, type(self.module).__name__,
               'add contiguous' if add.is_contiguous() else 'add strided')] += 1
    return _fwd(self, x, add, first)


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--lo', type=int, default=9)
    p.add_argument('--hi', type=int, default=24)
    p.add_argument('--batch', type=int, default=40)
    a = p.parse_args()
    am.Operation.forward = forward
    dev = torch.device('cuda')
    model = am.amoebanetd(num_classes=1000, num_layers=18, num_filters=256).to(dev)
    layers = list(model.children())
    head = torch.nn.Sequential(*layers[:a.lo])
    part = torch.nn.Sequential(*layers[a.lo:a.hi])
    with use_skip_tracker(SkipTracker()):
        with torch.no_grad():
            x = head(torch.randn(a.batch, 3, 224, 224, device=dev))
        COUNT.clear()
        x = tuple(t.detach().requires_grad_(True) for t in x) if isinstance(x, tuple) else x
        part(x)
    for k, v in sorted(COUNT.items(), key=lambda kv: -kv[1]):
        print(v, k)


if __name__ == '__main__':
    main()
