"""Where the first training step's time goes (host profile of step 1 vs step 2).

Builds the bench model on one GPU, runs one full step under cProfile (synchronised), then a
second step for comparison, and prints the top cumulative host functions of the first.

    python benchmarks/first_step.py --model amoebanet
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    p = argparse.ArgumentParser()
    p.add_argument('--model', choices=['unet', 'amoebanet'], default='amoebanet')
    p.add_argument('--top', type=int, default=40)
    args = p.parse_args()
    from torchgpipe_amd.models import amoebanetd, unet
    from torchgpipe_amd.parallel import PipelineStage
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    t0 = time.time()
    with torch.device('meta'):
        model = (amoebanetd(1000, 18, 256) if args.model == 'amoebanet'
                 else unet(depth=5, num_convs=5, base_channels=64))
    batch, chunks = (640, 32) if args.model == 'amoebanet' else (80, 2)
    shape = (3, 224, 224) if args.model == 'amoebanet' else (3, 192, 192)
    stage = PipelineStage(model, [len(model)], device=dev, chunks=chunks,
                          checkpoint='except_last')
    opt = torch.optim.SGD(stage.parameters(), lr=0.1)
    x = torch.rand(batch, *shape, device=dev)
    if args.model == 'amoebanet':
        tgt = torch.randint(1000, (batch,), device=dev)
        loss_fn = F.cross_entropy
    else:
        tgt = torch.ones(batch, 1, 192, 192, device=dev)
        loss_fn = F.binary_cross_entropy_with_logits
    torch.cuda.synchronize()
    print(f'build {time.time() - t0:.2f}s', flush=True)

    def step() -> None:
        stage.train_step(x, tgt, loss_fn)
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize()

    from torchgpipe_amd.ops import _ext
    before = set(_ext.require().conv_gemm_plans_export().splitlines())
    print(f'plans loaded {len(before)}', flush=True)
    prof = cProfile.Profile()
    t1 = time.time()
    prof.enable()
    step()
    prof.disable()
    print(f'step 1 {time.time() - t1:.2f}s', flush=True)
    new = sorted(set(_ext.require().conv_gemm_plans_export().splitlines()) - before)
    print(f'plans tuned in step 1: {len(new)}', flush=True)
    for line in new:
        print('  new plan:', line)
    t2 = time.time()
    step()
    print(f'step 2 {time.time() - t2:.2f}s', flush=True)
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats('tottime').print_stats(args.top)
    print(s.getvalue())


if __name__ == '__main__':
    main()
