"""Run one Winograd conv shape repeatedly (for rocprofv3 counter collection).

    python benchmarks/conv_probe.py --shape 40 128 128 96 --op fwd --iters 20
    (fwd / wgrad: F(2x2) kernels; fwd4 / wgrad4: fused F(4x4); fwd4nf / wgrad4nf: non-fused)
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchgpipe_amd.ops import _ext  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--shape', type=int, nargs=4, default=[40, 128, 128, 96], help='N C K H')
    p.add_argument('--op', choices=['fwd', 'wgrad', 'fwd4', 'wgrad4', 'fwd4nf', 'wgrad4nf'],
                   default='fwd')
    p.add_argument('--iters', type=int, default=20)
    a = p.parse_args()
    n, c, k, h = a.shape
    ops = _ext.require()
    x = torch.randn(n, c, h, h, device='cuda')
    w = torch.randn(k, c, 3, 3, device='cuda')
    dy = torch.randn(n, k, h, h, device='cuda')
    u = ops.wino_weight(w, False)
    u4 = ops.wino4_weight(w, False)
    for _ in range(a.iters):
        if a.op == 'fwd':
            ops.wino_conv(x, u, None, k, -1, 0)
        elif a.op == 'fwd4':
            ops.wino4_conv(x, u4, None, k, 6, 0)
        elif a.op == 'fwd4nf':
            ops.wino4_conv(x, u4, None, k, 14, 0)
        elif a.op == 'wgrad4':
            ops.wino4_wgrad(x, dy, 0, 0)
        elif a.op == 'wgrad4nf':
            ops.wino4_wgrad(x, dy, 0, 1)
        else:
            ops.wino_wgrad(x, dy, 0)
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
