"""Run one batched-GEMM Winograd convolution shape repeatedly (for rocprofv3 traces / PMC).

    python benchmarks/bg_probe.py --shape 16 1024 1024 12 --kind 4 --bn 0 --iters 10
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.ops import _ext  # noqa: E402


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--shape', type=int, nargs=4, required=True, help='N C K H')
    p.add_argument('--kind', type=int, default=4)
    p.add_argument('--bn', type=int, default=0)
    p.add_argument('--splits', type=int, default=0)
    p.add_argument('--iters', type=int, default=10)
    a = p.parse_args()
    n, c, k, h = a.shape
    dev = torch.device('cuda', 0)
    ops = _ext.require(torch.empty(0, device=dev))
    x = torch.randn(n, c, h, h, device=dev)
    w = torch.randn(k, c, 3, 3, device=dev) / (3 * c ** 0.5)
    wb = ops.bg_weight(w, False, a.kind)
    for _ in range(a.iters):
        ops.bg_conv(x, wb, None, k, a.bn, a.splits, a.kind)
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
