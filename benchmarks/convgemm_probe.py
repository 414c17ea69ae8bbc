"""Run one implicit-GEMM convolution launch repeatedly (for rocprofv3 counters).

    python benchmarks/convgemm_probe.py --x 20 1024 28 28 --co 256 --mode fwd --iters 10
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--x', type=int, nargs=4, required=True)
    p.add_argument('--co', type=int, required=True)
    p.add_argument('--k', type=int, nargs=2, default=[1, 1])
    p.add_argument('--stride', type=int, default=1)
    p.add_argument('--mode', choices=['fwd', 'bwd', 'wgrad'], default='fwd')
    p.add_argument('--iters', type=int, default=10)
    p.add_argument('--miopen', action='store_true', help='time MIOpen (F.conv2d) instead')
    p.add_argument('--force', type=int, nargs=2, default=None, metavar=('CFG', 'SPLITS'),
                   help='launch plan: tile config and (at most) this many reduction splits')
    a = p.parse_args()
    from torchgpipe_amd.ops import _ext
    ops = _ext.require()
    if a.force:
        ops.conv_gemm_force_cfg(*a.force)
    n, c, h, w = a.x
    kh, kw = a.k
    x = torch.randn(n, c, h, w, device='cuda')
    wt = torch.randn(a.co, c, kh, kw, device='cuda') * 0.05
    geo = [kh, kw, a.stride, a.stride, (kh - 1) // 2, (kw - 1) // 2, 0, 0]
    z = ops.conv_gemm_forward(x, wt, geo, True)
    dz = torch.randn_like(z)
    if a.miopen:
        import torch.nn.functional as F
        pad = (geo[4], geo[5])
        for _ in range(a.iters):
            if a.mode == 'fwd':
                F.conv2d(x, wt, stride=a.stride, padding=pad)
            else:
                torch.ops.aten.convolution_backward(
                    dz, x, wt, None, [a.stride] * 2, list(pad), [1, 1], False, [0, 0], 1,
                    [a.mode == 'bwd', a.mode == 'wgrad', False])
        torch.cuda.synchronize()
        return
    for _ in range(a.iters):
        if a.mode == 'fwd':
            ops.conv_gemm_forward(x, wt, geo, True)
        elif a.mode == 'bwd':
            ops.conv_gemm_backward_data(dz, x, wt, geo, True)
        else:
            ops.conv_gemm_backward_weight(dz, x, wt, geo, True)
    torch.cuda.synchronize()


if __name__ == '__main__':
    main()
