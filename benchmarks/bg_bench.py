"""Batched-GEMM Winograd F(4x4) (``bg_conv``) vs the shipped F(4x4)/F(2x2) kernels.

Times forward convolutions of the deep U-Net shapes at pipeline micro-batch sizes (16 at
pipeline-2/8, 32 at pipeline-4, 40 at pipeline-1) with HIP events: the kernels
``ops/conv.py`` dispatches today (weights pre-transformed, as in a pipeline step) against
``bg_conv`` at its planned tile and at every N-tile width.

    python benchmarks/bg_bench.py --out profiles/r3/bg_bench.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from torchgpipe_amd.ops import _ext  # noqa: E402
from torchgpipe_amd.ops.conv import _conv, _TransformCache  # noqa: E402

SHAPES = [  # (N, C, K, H)
    (16, 256, 512, 24), (16, 512, 512, 24), (16, 512, 1024, 12), (16, 1024, 1024, 12),
    (16, 1024, 2048, 6), (16, 2048, 2048, 6), (16, 2048, 512, 12), (16, 1024, 256, 24),
    (16, 512, 256, 24), (16, 256, 256, 48),
    (32, 1024, 1024, 12), (32, 2048, 2048, 6), (32, 512, 512, 24),
    (40, 1024, 1024, 12), (40, 2048, 2048, 6), (40, 512, 512, 24), (40, 256, 256, 48),
]


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    times = []
    for _ in range(iters):
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        times.append(e0.elapsed_time(e1))
    times.sort()
    return times[len(times) // 2]


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--iters', type=int, default=15)
    p.add_argument('--out', default=None)
    p.add_argument('--shapes', default=None,
                   help="'N,C,K,H;...' instead of the built-in U-Net shapes")
    a = p.parse_args()
    shapes = SHAPES if a.shapes is None else \
        [tuple(int(v) for v in part.split(',')) for part in a.shapes.split(';')]
    dev = torch.device('cuda', 0)
    ops = _ext.require(torch.empty(0, device=dev))
    rows = []
    for n, c, k, h in shapes:
        torch.manual_seed(0)
        x = torch.randn(n, c, h, h, device=dev)
        w = torch.randn(k, c, 3, 3, device=dev) / (3 * c ** 0.5)
        flops = 2.0 * n * k * c * 9 * h * h
        cache = _TransformCache()
        cur = timed(lambda: _conv(x, cache, w, None, False), a.iters)
        ref = torch.nn.functional.conv2d(x, w, padding=1)
        row = {'shape': [n, c, k, h], 'current_ms': round(cur, 4),
               'current_tflops': round(flops / cur / 1e9, 1)}
        for kind in (4, 2):
            wb = ops.bg_weight(w, False, kind)
            for waves, bn, sub in [(0, 0, 0)] + [(4, b, 1) for b in (48, 64, 96, 128)]:
                tag = f'f{kind}_{"auto" if not waves else f"{waves}x{bn}s{sub}"}'
                got = ops.bg_conv(x, wb, None, k, bn, 0, kind, waves, sub)
                err = ((got - ref).norm() / ref.norm()).item()
                if err > 1e-4:
                    raise SystemExit(f'{tag} {n, c, k, h}: relative error {err:.2e}')
                ms = timed(lambda: ops.bg_conv(x, wb, None, k, bn, 0, kind, waves, sub), a.iters)
                row[tag] = round(ms, 4)
            best = min((v, t) for t, v in row.items() if t.startswith(f'f{kind}_'))
            row[f'f{kind}_best'] = best[1]
        row['f4_auto_tflops'] = round(flops / row['f4_auto'] / 1e9, 1)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
