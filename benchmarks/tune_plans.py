"""Measure the implicit-GEMM convolution plans of the benchmark models and save them.

Runs one training forward + backward of U-Net(5,64) and AmoebaNet-D(18,256) on one GPU at
every micro-batch size the speed benchmarks use (``bench.py``'s experiment tables: the
micro-batch is global batch / chunks), so the autotuner in ``csrc/convbn.cpp`` measures
every convolution shape those runs meet, then writes the plan table.  The package loads
``torchgpipe_amd/tuned/conv_gemm_mi355x.txt`` at start-up, so benchmark processes on a
fresh machine skip the per-shape find (AmoebaNet's first step: seconds of candidate
timing per rank).

    python benchmarks/tune_plans.py --out torchgpipe_amd/tuned/conv_gemm_mi355x.txt
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

UNET_MICRO = (40, 16, 32)       # pipeline-1 80/2, -2 512/32 and -8 640/40, -4 512/16
AMOEBA_MICRO = (20, 40, 36)     # n1m32 640/32, n2/n8 1280/32, n4 1152/32


def run(model: torch.nn.Module, micro: int, shape, target_fn) -> None:
    x = torch.rand(micro, *shape, device='cuda')
    out = model(x)
    target_fn(out).backward()
    model.zero_grad(set_to_none=True)


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument('--out', required=True)
    p.add_argument('--models', default='amoebanet,unet')
    p.add_argument('--merge', action='store_true',
                   help='seed from the shipped table and measure only the shapes it lacks')
    args = p.parse_args()
    if not args.merge:
        os.environ['TGPIPE_CG_DB'] = '0'  # measure, do not seed from the shipped table
    from torchgpipe_amd.models import amoebanetd, unet
    from torchgpipe_amd.ops import _ext
    _ext.require()
    t0 = time.time()
    if 'amoebanet' in args.models:
        model = amoebanetd(num_classes=1000, num_layers=18, num_filters=256).cuda().train()
        for micro in AMOEBA_MICRO:
            run(model, micro, (3, 224, 224),
                lambda o: F.cross_entropy(o, torch.zeros(o.shape[0], dtype=torch.long,
                                                         device=o.device)))
            print(f'amoebanet micro-batch {micro}: {time.time() - t0:.1f}s', flush=True)
        del model
    if 'unet' in args.models:
        model = unet(depth=5, num_convs=5, base_channels=64, input_channels=3,
                     output_channels=1).cuda().train()
        for micro in UNET_MICRO:
            run(model, micro, (3, 192, 192), lambda o: o.float().square().mean())
            print(f'unet micro-batch {micro}: {time.time() - t0:.1f}s', flush=True)
        del model
    torch.cuda.synchronize()
    n = _ext.save_plans(args.out)
    print(f'{n} plans -> {args.out}', flush=True)


if __name__ == '__main__':
    main()
