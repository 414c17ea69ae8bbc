"""ResNet-101's 128-channel 3x3 layers (28^2) on the batched-GEMM Winograd (``bg_conv``)
instead of the fused F(4x4) kernel: forward and backward-data per micro-batch size, with
``ops/conv.py`` ``BG_MIN_CHANNELS`` at 256 (shipped) and 128.

    python benchmarks/diag/bg_min_channels_probe.py --out gpurun_out/bg_min_channels.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.ops import conv as conv_mod  # noqa: E402

SHAPES = [(22, 128, 28), (36, 128, 28), (110, 128, 28), (15, 128, 28), (22, 64, 56),
          (110, 64, 56)]


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
    rows = []
    for n, c, hw in SHAPES:
        x = torch.randn(n, c, hw, hw, device=dev)
        wt = torch.randn(c, c, 3, 3, device=dev) / (3 * c ** 0.5)
        row = {'shape': [n, c, c, hw, hw]}
        for mc in (256, c):
            conv_mod.BG_MIN_CHANNELS = mc
            cache = conv_mod._TransformCache()
            for flip in (False, True):
                def run(flip=flip, cache=cache):
                    return conv_mod._conv(x, cache, wt, None, flip)
                row[f'min{mc}_{"dgrad" if flip else "fwd"}_us'] = round(timed(run), 2)
        conv_mod.BG_MIN_CHANNELS = 256
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, 'w') as f:
            json.dump(rows, f, indent=1)


if __name__ == '__main__':
    main()
