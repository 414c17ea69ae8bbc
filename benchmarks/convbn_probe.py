"""One fused ReLU -> Conv -> BatchNorm op of AmoebaNet-D repeatedly, forward + backward on one
stream (for rocprofv3 --kernel-trace: every kernel of the op without the cell streams'
overlap inflating its duration).

    python benchmarks/convbn_probe.py --x 40 1024 7 7 --co 1024 --iters 10
"""
import argparse
import os
import sys

import torch
from torch import nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--x', type=int, nargs=4, required=True, metavar=('N', 'C', 'H', 'W'))
    p.add_argument('--co', type=int, required=True)
    p.add_argument('--k', type=int, nargs=2, default=[1, 1])
    p.add_argument('--iters', type=int, default=10)
    a = p.parse_args()
    from torchgpipe_amd.ops.convbn import ReLUConvBN
    n, c, h, w = a.x
    pad = ((a.k[0] - 1) // 2, (a.k[1] - 1) // 2)
    op = ReLUConvBN(nn.ReLU(), nn.Conv2d(c, a.co, tuple(a.k), padding=pad, bias=False),
                    nn.BatchNorm2d(a.co)).cuda()
    x = torch.randn(n, c, h, w, device='cuda', requires_grad=True)
    dy = None
    for _ in range(a.iters):
        y = op(x)
        if dy is None:
            dy = torch.randn_like(y)
        y.backward(dy)
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
