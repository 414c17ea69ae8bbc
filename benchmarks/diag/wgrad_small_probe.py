"""F(4x4) weight-gradient variants (0 fused f32, 1 non-fused f32, 2 split-bf16 batched GEMM)
at ResNet-101's pipeline micro-batches, where ``ops/conv.py`` ``_wgrad_f4_variant`` keeps
layers under 512 channels on the fused kernel.

    python benchmarks/diag/wgrad_small_probe.py --out gpurun_out/wgrad_small_probe.json
"""
import argparse
import json

import torch

from torchgpipe_amd.ops import _ext

SHAPES = [  # (N, C, K, H, W)
    (22, 256, 256, 14, 14), (36, 256, 256, 14, 14), (15, 256, 256, 14, 14),
    (22, 128, 128, 28, 28), (36, 128, 128, 28, 28), (22, 512, 512, 7, 7),
    (36, 512, 512, 7, 7), (110, 256, 256, 14, 14), (110, 128, 128, 28, 28),
    # U-Net(5, 64)'s 256-channel level (48^2) at the p1 / p4 / p8 micro-batches
    (40, 256, 256, 48, 48), (40, 512, 256, 48, 48), (32, 256, 256, 48, 48),
    (16, 256, 256, 48, 48), (16, 512, 256, 48, 48),
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
    for n, c, k, h, w in SHAPES:
        x = torch.randn(n, c, h, w, device=dev)
        dy = torch.randn(n, k, h, w, device=dev)
        ref = ops.wino4_wgrad(x, dy, 0, 0, None).double()
        row = {'shape': [n, c, k, h, w]}
        for v in (0, 1, 2):
            def run(v=v):
                return ops.wino4_wgrad(x, dy, 0, v, None)
            err = ((run().double() - ref).norm() / ref.norm()).item()
            row[f'v{v}_us'] = round(timed(run), 2)
            row[f'v{v}_rel_vs_v0'] = err
        row['f2_mfma_us'] = round(timed(lambda: ops.wino_wgrad(x, dy, 0, -1, None)), 2)
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
