"""Does the caching allocator still call hipMalloc / hipFree in steady-state steps?
ResNet-101 pipeline-1 (bench.py's configuration, lanes on) through PipelineStage: device
allocation / free counts per step after warm-up.

    python benchmarks/diag/alloc_probe.py --model resnet --steps 4
"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import resnet101, unet  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument('--model', choices=['resnet', 'unet'], default='resnet')
    p.add_argument('--steps', type=int, default=4)
    a = p.parse_args()
    dev = torch.device('cuda', 0)
    if a.model == 'resnet':
        model, batch, chunks, shape = resnet101(num_classes=1000), 220, 2, (3, 224, 224)
        target = torch.randint(0, 1000, (batch,), device=dev)
        loss_fn = F.cross_entropy
    else:
        model, batch, chunks, shape = unet(depth=5, num_convs=5, base_channels=64), 80, 2, \
            (3, 192, 192)
        target = torch.zeros(batch, 1, 192, 192, device=dev)
        loss_fn = F.binary_cross_entropy_with_logits
    stage = PipelineStage(model, [len(model)], device=dev, chunks=chunks,
                          checkpoint='except_last', overlap_recompute=True,
                          overlap_forward=True)
    x = torch.rand(batch, *shape, device=dev)
    opt = torch.optim.SGD(list(stage.parameters()), lr=0.1)
    for k in range(3 + a.steps):
        before = torch.cuda.memory_stats(dev)
        stage.train_step(x, target, loss_fn)
        opt.step()
        opt.zero_grad(set_to_none=True)
        torch.cuda.synchronize(dev)
        after = torch.cuda.memory_stats(dev)
        keys = ['num_device_alloc', 'num_device_free', 'num_alloc_retries', 'num_sync_all_streams']
        print(f'step {k}:', {kk: after.get(kk, 0) - before.get(kk, 0) for kk in keys},
              'reserved GiB', round(after['reserved_bytes.all.current'] / 2**30, 2), flush=True)


if __name__ == '__main__':
    main()
