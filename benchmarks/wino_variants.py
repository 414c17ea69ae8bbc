"""Time the Winograd forward kernel variants on U-Net conv shapes (and check them).

    python benchmarks/wino_variants.py --variants 0 2
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchgpipe_amd.ops import _ext  # noqa: E402

SHAPES = [  # N, C, K, H
    (40, 64, 64, 192), (16, 64, 64, 192), (16, 128, 128, 96), (16, 256, 256, 48),
    (16, 512, 512, 24), (16, 1024, 1024, 12), (16, 2048, 2048, 6), (16, 2048, 1024, 6),
    (16, 128, 64, 192), (40, 128, 32, 192), (40, 32, 32, 192), (16, 128, 32, 192),
    (16, 32, 32, 192), (3, 70, 130, 13),
    # the micro-batch of the 1-GPU bench (B=80, 2 chunks)
    (40, 128, 128, 96), (40, 256, 256, 48), (40, 512, 512, 24), (40, 1024, 1024, 12),
    (40, 2048, 2048, 6),
]


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--variants', type=int, nargs='+', default=[0, 2])
    p.add_argument('--iters', type=int, default=20)
    p.add_argument('--out', default=None)
    p.add_argument('--splits', type=int, nargs='+', default=[0],
                   help='split-K counts to time per variant (0: the planner picks)')
    p.add_argument('--shape', type=int, nargs=4, action='append', default=None,
                   help='N C K H (repeatable; default: the built-in table)')
    a = p.parse_args()
    ops = _ext.require()
    rows = []
    for n, c, k, h in (a.shape or SHAPES):
        torch.manual_seed(0)
        x = torch.randn(n, c, h, h, device='cuda')
        w = torch.randn(k, c, 3, 3, device='cuda') / (3 * c ** 0.5)
        u = ops.wino_weight(w, False)
        u4 = ops.wino4_weight(w, False) if max(a.variants) >= 4 else None
        ref = F.conv2d(x.double(), w.double(), padding=1)
        row = {'shape': [n, c, k, h]}
        for v, sp in [(v, sp) for v in a.variants for sp in a.splits]:
            # variants >= 4 = Winograd F(4x4,3x3) (winograd_f4.hip; 8-10 are timing
            # ablations with wrong results), the rest F(2x2,3x3)
            def run():  # noqa: E306
                if v >= 4:
                    return ops.wino4_conv(x, u4, None, k, v, sp)
                return ops.wino_conv(x, u, None, k, v, sp)
            y = run()
            err = ((y.double() - ref).abs().max() / (ref.abs().max() + 1e-12)).item()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(3):
                run()
            s.record()
            for _ in range(a.iters):
                run()
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / a.iters
            tf = 2.0 * n * k * c * 9 * h * h / ms / 1e9
            tag = f'v{v}' + (f's{sp}' if sp else '')
            row[tag] = {'ms': round(ms, 4), 'direct_tflops': round(tf, 1), 'rel_err': err}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        json.dump(rows, open(a.out, 'w'), indent=1)


if __name__ == '__main__':
    main()
