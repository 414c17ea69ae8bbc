"""Which parameters of a ResNet partition on lanes get wrong gradients, and does taking the
MIOpen stem convolution off the lanes' concurrency change it?  Several trials per variant;
prints every parameter whose gradient is off by more than 1e-4 of its largest element."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from torchgpipe_amd.models.resnet import build_resnet  # noqa: E402
from torchgpipe_amd.ops import fusion  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402


def trial(checkpoint, fwd, rec, seed):
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = build_resnet([1, 1, 1, 1], num_classes=10)
    a, b = copy.deepcopy(base).to(dev), copy.deepcopy(base).to(dev)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       overlap_recompute=rec, overlap_forward=fwd)
    gen = torch.Generator(device=dev).manual_seed(seed)
    bad = []
    for step in range(3):
        x = torch.rand(16, 3, 64, 64, device=dev, generator=gen)
        y = torch.randint(10, (16,), device=dev, generator=gen)
        for p in list(a.parameters()) + list(b.parameters()):
            p.grad = None
        sa.train_step(x, y, F.cross_entropy)
        sb.train_step(x, y, F.cross_entropy)
        torch.cuda.synchronize()
        for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
            err = (pb.grad - pa.grad).abs().max().item() / (pa.grad.abs().max().item() + 1e-12)
            if err > 1e-4:
                bad.append((step, n, round(err, 5)))
    return bad


for variant in ('miopen_stem', 'native_stem'):
    if variant == 'native_stem':
        fusion.STRIDED_FUSED = fusion.STRIDED_FUSED | {(3, 64, (7, 7), (2, 2), (3, 3), 64)}
    for checkpoint in ('always', 'except_last'):
        for fwd, rec in ((True, True), (True, False), (False, True)):
            for seed in range(3):
                bad = trial(checkpoint, fwd, rec, 5 + seed)
                print(variant, checkpoint, f'fwd={fwd} rec={rec} seed={seed}',
                      'OK' if not bad else bad[:6], flush=True)
