"""Split-bf16 batched-GEMM Winograd (``bg_conv``) at ResNet-101's pipeline micro-batches:
the GEMM tile width (BN 64 / 96 / 128) per shape, forward and backward-data, with the
automatic choice for comparison.  Small tile counts leave the 128-wide tile's grid under
one workgroup per CU.

    python benchmarks/diag/bg_tile_probe.py --out gpurun_out/bg_tile_probe.json
"""
import argparse
import json

import torch

from torchgpipe_amd.ops import _ext

SHAPES = [  # (N, C, K, H, W, kind): ResNet-101 3x3 layers at the p4 / p8 / p2 micro-batches
    (22, 256, 256, 14, 14, 4), (22, 512, 512, 7, 7, 2), (22, 128, 128, 28, 28, 4),
    (36, 256, 256, 14, 14, 4), (36, 512, 512, 7, 7, 2), (36, 128, 128, 28, 28, 4),
    (15, 256, 256, 14, 14, 4), (15, 512, 512, 7, 7, 2),
]


def timed(fn, reps=40):
    for _ in range(5):
        fn()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(reps):
        fn()
    ev[1].record()
    ev[1].synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / reps


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--out', default=None)
    a = p.parse_args()
    dev = torch.device('cuda')
    ops = _ext.require(torch.empty(1, device=dev))
    rows = []
    for n, c, k, h, w, kind in SHAPES:
        for flip in (False, True):
            cin, cout = (k, c) if flip else (c, k)
            x = torch.randn(n, cin, h, w, device=dev)
            wt = torch.randn(k, c, 3, 3, device=dev)
            u = ops.bg_weight(wt, flip, kind, emu=1)
            row = {'shape': [n, c, k, h, w], 'kind': kind, 'flip': flip}
            for bn in (0, 64, 96, 128):  # 0: the automatic width (bn / waves given: forced)
                def run(bn=bn):
                    return ops.bg_conv(x, u, None, cout, bn, 0, kind, 4 if bn else 0, 0, emu=1)
                row[f'bn{bn}_us'] = round(timed(run), 2)
            rows.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
