"""Implicit-GEMM convolutions vs the 1x1 convolution of the same GEMM dimensions.

A kh x kw convolution with C input channels is the GEMM of a 1x1 convolution with C*kh*kw
input channels; the difference in time is what the tap gather (index math, unaligned
loads, padding checks) costs.  Times forward / backward-data / weight-gradient of each
pair with the tuned plans (HIP events, median of repeats).

    python benchmarks/gemm_equiv.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PAIRS = [  # n, c, h, co, kh, kw
    (20, 64, 28, 64, 1, 7), (20, 64, 28, 64, 7, 1), (20, 128, 14, 128, 1, 7),
    (20, 128, 14, 128, 7, 1), (20, 256, 7, 256, 1, 7), (20, 256, 7, 256, 7, 1),
]


def timed(fn, iters: int = 20) -> float:
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return 1000.0 * s.elapsed_time(e) / iters


def run(ops, n: int, c: int, h: int, co: int, kh: int, kw: int) -> dict:
    x = torch.randn(n, c, h, h, device='cuda')
    wt = torch.randn(co, c, kh, kw, device='cuda') * 0.05
    geo = [kh, kw, 1, 1, (kh - 1) // 2, (kw - 1) // 2, 0, 0]
    z = ops.conv_gemm_forward(x, wt, geo, True)
    dz = torch.randn_like(z)
    return {
        'fwd': timed(lambda: ops.conv_gemm_forward(x, wt, geo, True)),
        'bwd': timed(lambda: ops.conv_gemm_backward_data(dz, x, wt, geo, True)),
        'wgrad': timed(lambda: ops.conv_gemm_backward_weight(dz, x, wt, geo, True)),
    }


def main() -> None:
    from torchgpipe_amd.ops import _ext
    ops = _ext.require()
    rows = []
    for n, c, h, co, kh, kw in PAIRS:
        taps = run(ops, n, c, h, co, kh, kw)
        flat = run(ops, n, c * kh * kw, h, co, 1, 1)
        gflop = 2.0 * n * co * c * kh * kw * h * h / 1e9
        row = {'shape': [n, c, h, co, kh, kw], 'gflop': round(gflop, 3),
               'taps_us': {k: round(v, 2) for k, v in taps.items()},
               'flat1x1_us': {k: round(v, 2) for k, v in flat.items()}}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if len(sys.argv) > 1:
        json.dump(rows, open(sys.argv[1], 'w'), indent=1)


if __name__ == '__main__':
    main()
