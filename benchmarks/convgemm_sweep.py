"""Device time of every implicit-GEMM launch plan (tile config x reduction splits) for a
few AmoebaNet-D convolution shapes (micro-batch 20: ``--micro-batch``) -- what the
autotuner chooses from.

    python benchmarks/convgemm_sweep.py --out profiles/convgemm_sweep.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = [  # N, Ci, H, Co, kh, kw
    (20, 1024, 7, 1024, 1, 1), (20, 4096, 7, 1024, 1, 1), (20, 256, 7, 256, 1, 7),
    (20, 512, 14, 512, 1, 1), (20, 256, 28, 256, 1, 1), (20, 1024, 28, 256, 1, 1),
    (20, 64, 28, 64, 1, 7), (20, 64, 28, 256, 1, 1),
]
CFG = {0: '64x64/4w', 1: '128x128/8w', 2: '128x128/4w', 3: '64x64/4w/sub4',
       4: '128x128/8w/sub2', 5: '128x128/4w/sub2', 6: '64x64/4w/sub2',
       7: 'emu 64x64/4w', 8: 'emu 128x128/4w', 9: 'emu 128x128/8w',
       10: 'emu 128x128/8w/single', 11: 'emu 64x64/4w/single'}
# ResNet-101's 1x1 / 3x3 shapes at its micro-batches (--set resnet; N from --micro-batch)
RESNET_SHAPES = [
    (22, 256, 56, 64, 1, 1), (22, 64, 56, 256, 1, 1), (22, 512, 28, 128, 1, 1),
    (22, 128, 28, 512, 1, 1), (22, 1024, 14, 256, 1, 1), (22, 256, 14, 1024, 1, 1),
    (22, 2048, 7, 512, 1, 1), (22, 512, 7, 2048, 1, 1), (22, 256, 14, 256, 3, 3),
    (22, 1024, 7, 2048, 1, 1), (22, 2048, 7, 1024, 1, 1),
]


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument('--reps', type=int, default=20)
    p.add_argument('--micro-batch', type=int, default=20, help='images per shape')
    p.add_argument('--out', default='')
    p.add_argument('--set', choices=['amoebanet', 'resnet'], default='amoebanet')
    a = p.parse_args()
    from torchgpipe_amd.ops import _ext
    ops = _ext.require()
    out = []
    for _, ci, h, co, kh, kw in (SHAPES if a.set == 'amoebanet' else RESNET_SHAPES):
        n = a.micro_batch
        x = torch.randn(n, ci, h, h, device='cuda')
        w = torch.randn(co, ci, kh, kw, device='cuda') * 0.05
        geo = [kh, kw, 1, 1, (kh - 1) // 2, (kw - 1) // 2, 0, 0]
        gflop = 2.0 * n * h * h * co * ci * kh * kw / 1e9
        for mode, name in enumerate(('fwd', 'bwd_data', 'wgrad')):
            r = ops.conv_gemm_sweep(mode, x, w, geo, a.reps)
            cands = sorted(([CFG[int(r[i])], int(r[i + 1]), round(r[i + 2], 2)]
                            for i in range(0, len(r), 3)), key=lambda c: c[2])
            row = {'shape': [n, ci, h, co, kh, kw], 'mode': name, 'gflop': round(gflop, 3),
                   'best_us': cands[0][2], 'best_tflops': round(gflop / cands[0][2] * 1e3, 1),
                   'top': cands[:6]}
            # the double- vs single-buffered 8-wave split-bf16 tile, each at its best split
            for cfg in (7, 9, 10, 11):
                mine = [c for c in cands if c[0] == CFG[cfg]]
                if mine:
                    row[f'cfg{cfg}_us'] = mine[0][2]
            out.append(row)
            print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(out, f, indent=1)


if __name__ == '__main__':
    main()
