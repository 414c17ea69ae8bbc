"""Pin down the ResNet-on-lanes gradient difference: plain vs plain (determinism), and the
recompute lanes with / without slotted running statistics, with / without the prefetched
recomputation, and with momentum left alone, on the seeds that differed."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from torchgpipe_amd.models.resnet import build_resnet  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402
from torchgpipe_amd import runstats  # noqa: E402


def trial(checkpoint, seed, variant):
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = build_resnet([1, 1, 1, 1], num_classes=10)
    a, b = copy.deepcopy(base).to(dev), copy.deepcopy(base).to(dev)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint)
    rec = variant != 'plain'
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       overlap_recompute=rec)
    if variant == 'lanes_noslots':
        sb._stat_slots = None
    gen = torch.Generator(device=dev).manual_seed(seed)
    out = []
    for step in range(3):
        x = torch.rand(16, 3, 64, 64, device=dev, generator=gen)
        y = torch.randint(10, (16,), device=dev, generator=gen)
        for p in list(a.parameters()) + list(b.parameters()):
            p.grad = None
        sa.train_step(x, y, F.cross_entropy)
        sb.train_step(x, y, F.cross_entropy)
        torch.cuda.synchronize()
        worst = max(((pb.grad - pa.grad).abs().max().item()
                     / (pa.grad.abs().max().item() + 1e-12), n)
                    for (n, pa), pb in zip(a.named_parameters(), b.parameters()))
        nbad = sum((pb.grad - pa.grad).abs().max().item()
                   > 1e-4 * (pa.grad.abs().max().item() + 1e-12)
                   for pa, pb in zip(a.parameters(), b.parameters()))
        bufd = max((bb.float() - ba.float()).abs().max().item()
                   for ba, bb in zip(a.buffers(), b.buffers()))
        out.append(f'step{step}: worst {worst[0]:.1e} {worst[1]} bad {nbad} buf {bufd:.1e}')
    return out


_orig_update = runstats.OrderedRunningStats.update
for checkpoint in ('except_last', 'always'):
    for seed in (6, 7):
        for variant in ('plain', 'lanes', 'lanes_noslots'):
            print(checkpoint, seed, variant, trial(checkpoint, seed, variant), flush=True)
