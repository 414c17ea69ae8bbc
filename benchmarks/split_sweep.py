"""Split-K sweep of the F(4x4) weight-gradient and fused forward kernels.

The host heuristics (``wino4_wgrad_splits`` / ``wino4_plan`` in csrc/winograd_f4.hip) ask
for >= 32 (weight gradient) / >= 16 (forward) reduction steps per split, which at
ResNet-101's 15-36-image micro-batches leaves most of the 256 CUs idle (14^2 x 256
channels at 22 images: 64 workgroups for 136 us, profiles/r5/rocprof/
resnet_p4_stage2_mb22.md).  This times every split count per shape (and the non-fused
weight-gradient variant) so the heuristic can be fitted to measurements.

    python benchmarks/split_sweep.py --out gpurun_out/split_sweep.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from torchgpipe_amd.ops import _ext  # noqa: E402

# N, C (input channels), K (output channels), H: ResNet-101's stride-1 3x3 convolutions at
# the reference's micro-batches (p2 15, p4 22, p8 36) and U-Net's at 16 / 40 images
SHAPES = [(n, c, c, h) for n in (15, 22, 36)
          for c, h in ((64, 56), (128, 28), (256, 14), (512, 7))] + [
    (40, 64, 64, 192), (40, 128, 128, 96), (40, 256, 256, 48), (16, 64, 64, 192),
    (16, 128, 128, 96), (16, 256, 256, 48), (16, 512, 512, 24), (40, 512, 512, 24),
    (16, 1024, 1024, 12), (40, 1024, 1024, 12), (40, 128, 32, 192), (40, 32, 32, 192),
]
SPLITS = (1, 2, 3, 4, 6, 8, 12, 16, 24, 32, 48, 64, 96, 128, 192, 256)
# batched-GEMM Winograd (bg_conv, split-bf16): ResNet's 14^2 / 7^2 layers and U-Net's deep ones
BG_SHAPES = [(n, c, c, h) for n in (15, 22, 36) for c, h in ((256, 14), (512, 7))] + [
    (40, 256, 256, 48), (40, 512, 512, 24), (40, 1024, 1024, 12), (16, 256, 256, 48),
    (16, 512, 512, 24), (16, 1024, 1024, 12), (16, 2048, 2048, 6), (110, 256, 256, 14),
    (110, 512, 512, 7)]
BG_SPLITS = (1, 2, 3, 4, 6, 8)


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


def bg_row(ops, n, c, k, h, iters):  # type: ignore[no-untyped-def]
    """Every (tile width, split count) of the batched-GEMM forward at one shape."""
    torch.manual_seed(0)
    kind = 2 if h < 8 else 4
    x = torch.randn(n, c, h, h, device='cuda')
    w = torch.randn(k, c, 3, 3, device='cuda') * 0.05
    a = ops.bg_weight(w, False, kind)
    ref = ops.bg_conv(x, a, None, k, 128, 1, kind, 4).double()
    res = {'auto': round(timed(lambda: ops.bg_conv(x, a, None, k, 0, 0, kind), iters), 4)}
    best = None
    for bn in (64, 96, 128):
        for s in BG_SPLITS:
            if s > -(-c // 16):
                break
            got = ops.bg_conv(x, a, None, k, bn, s, kind, 4).double()
            err = ((got - ref).abs().max() / ref.abs().max()).item()
            assert err < 1e-3, (n, c, k, h, bn, s, err)
            ms = timed(lambda: ops.bg_conv(x, a, None, k, bn, s, kind, 4), iters)
            res[f'{bn}/{s}'] = round(ms, 4)
            if best is None or ms < res[best]:
                best = f'{bn}/{s}'
    res['best'] = best
    return {'shape': [n, c, k, h], 'bg': res}


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--iters', type=int, default=20)
    p.add_argument('--out', default=None)
    p.add_argument('--ops', default='wgrad,fwd', help="any of wgrad, fwd, bg")
    p.add_argument('--shape', type=int, nargs=4, action='append', default=None,
                   help='N C K H (repeatable; default: the built-in table)')
    a = p.parse_args()
    ops = _ext.require()
    rows = []
    if 'bg' in a.ops:
        for n, c, k, h in BG_SHAPES:
            rows.append(bg_row(ops, n, c, k, h, a.iters))
            print(json.dumps(rows[-1]), flush=True)
    for n, c, k, h in (a.shape or SHAPES):
        if 'wgrad' not in a.ops and 'fwd' not in a.ops:
            break
        torch.manual_seed(0)
        x = torch.randn(n, c, h, h, device='cuda')
        dy = torch.randn(n, k, h, h, device='cuda')
        w = torch.randn(k, c, 3, 3, device='cuda') * 0.05
        row = {'shape': [n, c, k, h]}
        steps_wg = (n * -(-h // 4) * -(-h // 4) + 3) // 4
        if 'wgrad' in a.ops and h >= 6:
            ref = ops.wino4_wgrad(x, dy, 1, 0).double()
            for var in (0, 1):
                best = None
                res = {'auto': round(timed(lambda: ops.wino4_wgrad(x, dy, 0, var), a.iters), 4)}
                for s in SPLITS:
                    if s > steps_wg:
                        break
                    got = ops.wino4_wgrad(x, dy, s, var).double()
                    err = ((got - ref).abs().max() / ref.abs().max()).item()
                    assert err < 1e-3, (n, c, k, h, var, s, err)  # fp32 summation orders
                    ms = timed(lambda: ops.wino4_wgrad(x, dy, s, var), a.iters)
                    res[str(s)] = round(ms, 4)
                    if best is None or ms < res[str(best)]:
                        best = s
                res['best'] = best
                row[f'wgrad_v{var}'] = res
        if 'fwd' in a.ops and h >= 8 and k < 256:
            u = ops.wino4_weight(w, False)
            steps = -(-c // 4)
            tiles = n * -(-h // 4) * -(-h // 4)
            blocks = -(-tiles // 32) * -(-k // 64)
            for var in (6, 7):
                ref = ops.wino4_conv(x, u, None, k, var, 1).double()
                res = {'auto': round(timed(lambda: ops.wino4_conv(x, u, None, k, var, 0),
                                           a.iters), 4)}
                best = None
                for s in SPLITS:
                    if s > steps:
                        break
                    got = ops.wino4_conv(x, u, None, k, var, s).double()
                    err = ((got - ref).abs().max() / ref.abs().max()).item()
                    assert err < 1e-3, (n, c, k, h, var, s, err)  # fp32 summation orders
                    ms = timed(lambda: ops.wino4_conv(x, u, None, k, var, s), a.iters)
                    res[str(s)] = round(ms, 4)
                    if best is None or ms < res[str(best)]:
                        best = s
                res['best'] = best
                res['blocks64'] = blocks
                row[f'fwd_v{var}'] = res
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
