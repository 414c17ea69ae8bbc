"""Which part of a BatchNorm partition on lanes changes its gradients?  Step by step,
the worst parameter-gradient and buffer differences against the one-stream schedule, for
forward lanes / recompute lanes / both, with and without slotted running statistics."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from torchgpipe_amd.models.resnet import build_resnet  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402


def run(fwd, rec, slots, checkpoint='except_last'):
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = build_resnet([1, 1, 1, 1], num_classes=10)
    a, b = copy.deepcopy(base).to(dev), copy.deepcopy(base).to(dev)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       overlap_recompute=rec, overlap_forward=fwd)
    if not slots:
        sb._stat_slots = None
        sb._lanes_ok = lambda: True
    gen = torch.Generator(device=dev).manual_seed(5)
    for step in range(3):
        x = torch.rand(16, 3, 64, 64, device=dev, generator=gen)
        y = torch.randint(10, (16,), device=dev, generator=gen)
        for p in list(a.parameters()) + list(b.parameters()):
            p.grad = None
        la = sa.train_step(x, y, F.cross_entropy)
        lb = sb.train_step(x, y, F.cross_entropy)
        torch.cuda.synchronize()
        worst = max(((pb.grad - pa.grad).abs().max().item()
                     / (pa.grad.abs().max().item() + 1e-12), n)
                    for (n, pa), pb in zip(a.named_parameters(), b.parameters()))
        bw = max(((bb.float() - ba.float()).abs().max().item(), n)
                 for (n, ba), bb in zip(a.named_buffers(), b.buffers()))
        print(f'fwd={fwd} rec={rec} slots={slots} step {step}: '
              f'loss {abs(la.item() - lb.item()):.2e} '
              f'grad {worst[0]:.2e} {worst[1]}  buffer {bw[0]:.2e} {bw[1]}', flush=True)


for fwd, rec, slots in [(False, True, True), (False, True, False), (True, False, True),
                        (True, True, True), (True, False, False)]:
    run(fwd, rec, slots)
