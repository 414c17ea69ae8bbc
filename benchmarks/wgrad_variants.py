"""Time the Winograd weight-gradient kernels (F(2x2) variants 0 / 2, F(4x4)) against MIOpen's wrw.

    python benchmarks/wgrad_variants.py --out gpurun_out/wgrad_variants.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchgpipe_amd.ops import _ext  # noqa: E402

SHAPES = [  # N, C, K, H
    (40, 64, 64, 192), (16, 64, 64, 192), (16, 128, 128, 96), (16, 256, 256, 48),
    (16, 512, 512, 24), (16, 1024, 1024, 12), (16, 2048, 2048, 6), (16, 2048, 1024, 6),
    (40, 128, 32, 192), (40, 32, 32, 192), (40, 256, 256, 48), (40, 1024, 1024, 12),
    (40, 128, 128, 96), (40, 512, 512, 24),
    (3, 70, 130, 13),
]


def timed(fn, iters):  # type: ignore[no-untyped-def]
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--iters', type=int, default=10)
    p.add_argument('--out', default=None)
    p.add_argument('--shape', type=int, nargs=4, action='append', default=None,
                   help='N C K H (repeatable; default: the built-in table)')
    p.add_argument('--all-f4', action='store_true', help='time F(4x4) below 8x8 planes too')
    a = p.parse_args()
    ops = _ext.require()
    rows = []
    for n, c, k, h in (a.shape or SHAPES):
        torch.manual_seed(0)
        x = torch.randn(n, c, h, h, device='cuda')
        dy = torch.randn(n, k, h, h, device='cuda')
        w0 = torch.zeros(k, c, 3, 3, device='cuda')

        def miopen():  # type: ignore[no-untyped-def]
            return torch.ops.aten.convolution_backward(dy, x, w0, None, [1, 1], [1, 1], [1, 1],
                                                       False, [0, 0], 1,
                                                       [False, True, False])[1]
        ref = torch.ops.aten.convolution_backward(
            dy.double(), x.double(), w0.double(), None, [1, 1], [1, 1], [1, 1], False, [0, 0],
            1, [False, True, False])[1]
        flops = 2.0 * n * k * c * 9 * h * h
        row = {'shape': [n, c, k, h], 'miopen_ms': round(timed(miopen, a.iters), 4)}
        for v in (0, 2):
            got = ops.wino_wgrad(x, dy, 0, v)
            err = ((got.double() - ref).abs().max() / ref.abs().max()).item()
            ms = timed(lambda: ops.wino_wgrad(x, dy, 0, v), a.iters)
            row[f'v{v}'] = {'ms': round(ms, 4), 'direct_tflops': round(flops / ms / 1e9, 1),
                            'rel_err': err}
        if h >= 8 or a.all_f4:
            for name, var in (('f4', 0), ('f4nf', 1), ('f4emu', 2)):
                got = ops.wino4_wgrad(x, dy, 0, var)
                err = ((got.double() - ref).abs().max() / ref.abs().max()).item()
                ms = timed(lambda: ops.wino4_wgrad(x, dy, 0, var), a.iters)
                row[name] = {'ms': round(ms, 4), 'direct_tflops': round(flops / ms / 1e9, 1),
                             'rel_err': err}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        json.dump(rows, open(a.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
