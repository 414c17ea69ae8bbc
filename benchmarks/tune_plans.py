"""Measure the implicit-GEMM convolution plans of the benchmark models and save them.

Runs one training forward + backward of U-Net(5,64), AmoebaNet-D(18,256) and ResNet-101
on one GPU at every micro-batch size the speed benchmarks use (``bench.py``'s experiment
tables: the micro-batch is global batch / chunks) with the autotuner of
``csrc/convbn.cpp`` switched on (``TGPIPE_CG_TUNE=1``), so it times every candidate plan
of every convolution shape those runs meet -- and, for backward-data, the library
convolution against the implicit GEMM -- then writes both tables.  Training processes
only *read* them (``torchgpipe_amd/tuned/``): no training step ever synchronises the host
to time kernels, and every rank of a pipeline runs the same plan for a shape.

    python benchmarks/tune_plans.py --out torchgpipe_amd/tuned/conv_gemm_mi355x.txt \
        --lib-out torchgpipe_amd/tuned/lib_dgrad_mi355x.txt
"""
import argparse
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

UNET_MICRO = (40, 16, 32)       # pipeline-1 80/2, -2 512/32 and -8 640/40, -4 512/16
AMOEBA_MICRO = (20, 40, 36, 96)  # n1m32 640/32, n2/n8 1280/32, n4 1152/32, n2m1 96/1
# pipeline-1 220/2, pipeline-2 3520/32, the reference's pipeline-4 5632/256 and -8 5400/150,
# its pipeline-2 25000/1667
RESNET_MICRO = (110, 22, 36, 15)


def run(model: torch.nn.Module, micro: int, shape, target_fn) -> None:
    x = torch.rand(micro, *shape, device='cuda')
    out = model(x)
    target_fn(out).backward()
    model.zero_grad(set_to_none=True)


def main() -> None:
    p = argparse.ArgumentParser(description=__doc__)
    p.add_argument('--out', required=True)
    p.add_argument('--lib-out', default=None, help='backward-data library-choice table')
    p.add_argument('--models', default='amoebanet,unet,resnet')
    p.add_argument('--merge', action='store_true',
                   help='seed from the shipped table and measure only the shapes it lacks')
    args = p.parse_args()
    os.environ['TGPIPE_CG_TUNE'] = '1'  # time candidates on first use (this script only)
    if not args.merge:
        os.environ['TGPIPE_CG_DB'] = '0'  # measure, do not seed from the shipped tables
        os.environ['TGPIPE_LIB_DGRAD_DB'] = '0'
    from torchgpipe_amd.models import amoebanetd, resnet101, unet
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
    if 'resnet' in args.models:
        model = resnet101(num_classes=1000).cuda().train()
        for micro in RESNET_MICRO:
            run(model, micro, (3, 224, 224),
                lambda o: F.cross_entropy(o, torch.zeros(o.shape[0], dtype=torch.long,
                                                         device=o.device)))
            print(f'resnet101 micro-batch {micro}: {time.time() - t0:.1f}s', flush=True)
        del model
    torch.cuda.synchronize()
    n = _ext.save_plans(args.out)
    print(f'{n} plans -> {args.out}', flush=True)
    if args.lib_out:
        n = _ext.save_lib_dgrad(args.lib_out)
        print(f'{n} library backward-data geometries -> {args.lib_out}', flush=True)


if __name__ == '__main__':
    main()
