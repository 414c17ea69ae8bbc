"""Two-stream cells over several SGD steps: at every step, compare the two-stream model B
with a one-stream copy C loaded with B's current parameters and buffers, so any difference
is the step's own (not divergence accumulated from earlier steps)."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import amoebanetd  # noqa: E402
from torchgpipe_amd.models.amoebanet import set_cell_streams  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402

dev = torch.device('cuda', 0)
torch.manual_seed(0)
b = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
set_cell_streams(b, True)
sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last')
ob = torch.optim.SGD(sb.parameters(), lr=0.05)
gen = torch.Generator(device=dev).manual_seed(13)
for step in range(5):
    c = copy.deepcopy(b)
    set_cell_streams(c, False)
    sc = PipelineStage(c, [len(c)], device=dev, chunks=4, checkpoint='except_last')
    x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
    y = torch.randint(10, (8,), device=dev, generator=gen)
    lb = sb.train_step(x, y, F.cross_entropy)
    lc = sc.train_step(x, y, F.cross_entropy)
    torch.cuda.synchronize()
    worst = max(((pb.grad - pc.grad).abs().max() / (pc.grad.abs().max() + 1e-12)).item()
                for pb, pc in zip(b.parameters(), c.parameters()))
    print(f'step {step}: loss {lb.item():.6f} vs {lc.item():.6f}, worst grad diff {worst:.1e}',
          flush=True)
    ob.step()
    ob.zero_grad(set_to_none=True)
