"""The strided Conv-BN(-ReLU) geometries where the fused native op beats MIOpen + the native
BatchNorm, timed per micro-batch size (``ops/fusion.py`` ``_strided_fused`` with
``STRIDED_CHOICE``): one ResNet-101 forward + backward per size, then the picks.

    python benchmarks/diag/strided_picks.py --batches 15 22 36 110
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import resnet101  # noqa: E402
from torchgpipe_amd.ops import fusion  # noqa: E402
from torchgpipe_amd.skip.tracker import SkipTracker, use_skip_tracker  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--batches', type=int, nargs='+', default=[15, 22, 36, 110])
    p.add_argument('--out', default=None)
    a = p.parse_args()
    fusion.STRIDED_CHOICE = True
    dev = torch.device('cuda')
    model = resnet101(num_classes=1000).to(dev)
    fusion.relink(model)
    rows = []
    for n in a.batches:
        fusion._STRIDED.clear()
        x = torch.randn(n, 3, 224, 224, device=dev)
        t = torch.randint(0, 1000, (n,), device=dev)
        with use_skip_tracker(SkipTracker()):
            F.cross_entropy(model(x), t).backward()
        torch.cuda.synchronize()
        for key, pick in fusion._STRIDED.items():
            shape, cout, k, s, pad = key[0], key[1], key[2], key[3], key[4]
            row = {'batch': n, 'in': shape[1], 'out': cout, 'kernel': list(k),
                   'stride': list(s), 'padding': list(pad), 'height': shape[2],
                   'relu': key[5], 'fused': pick}
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
