"""Weight-gradient stream over several SGD steps: per-step gradient difference of the
stem convolution against the one-stream model, per configuration (debug probe)."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import amoebanetd  # noqa: E402
from torchgpipe_amd.models.amoebanet import set_cell_streams  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402


def run(streams: bool, overlap: bool, wgrad: bool, sync: bool) -> None:
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    set_cell_streams(b, streams)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint='except_last')
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint='except_last',
                       overlap_recompute=overlap, wgrad_stream=wgrad)
    oa = torch.optim.SGD(sa.parameters(), lr=0.05)
    ob = torch.optim.SGD(sb.parameters(), lr=0.05)
    gen = torch.Generator(device=dev).manual_seed(13)
    out = []
    for _ in range(4):
        x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
        y = torch.randint(10, (8,), device=dev, generator=gen)
        sa.train_step(x, y, F.cross_entropy)
        sb.train_step(x, y, F.cross_entropy)
        if sync:
            torch.cuda.synchronize()
        worst = 0.0
        for pa, pb in zip(a.parameters(), b.parameters()):
            d = ((pb.grad - pa.grad).abs().max() / (pa.grad.abs().max() + 1e-12)).item()
            worst = max(worst, d)
        pdiff = max(((pb - pa).abs().max() / (pa.abs().max() + 1e-12)).item()
                    for pa, pb in zip(a.parameters(), b.parameters()))
        out.append((f'{worst:.1e}', f'{pdiff:.1e}'))
        oa.step()
        ob.step()
        oa.zero_grad(set_to_none=True)
        ob.zero_grad(set_to_none=True)
    print(f'streams={streams} overlap={overlap} wgrad={wgrad} sync={sync}: '
          f'(grad diff, param diff) per step {out}', flush=True)


for cfg in [(False, False, False, False), (False, False, True, False), (False, False, True, True),
            (False, True, True, False), (True, False, True, False), (True, True, False, False)]:
    run(*cfg)
