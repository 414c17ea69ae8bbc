"""Which gradients differ with the weight-gradient stream (debug probe, one GPU)."""
import copy
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from torchgpipe_amd.models import amoebanetd  # noqa: E402
from torchgpipe_amd.models.amoebanet import set_cell_streams  # noqa: E402
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402


def run(streams: bool, overlap: bool, wgrad: bool, chunks: int, checkpoint: str) -> None:
    dev = torch.device('cuda', 0)
    torch.manual_seed(0)
    base = amoebanetd(num_classes=10, num_layers=3, num_filters=16)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    set_cell_streams(b, streams)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=chunks, checkpoint=checkpoint)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=chunks, checkpoint=checkpoint,
                       overlap_recompute=overlap, wgrad_stream=wgrad)
    gen = torch.Generator(device=dev).manual_seed(13)
    x = torch.rand(8, 3, 224, 224, device=dev, generator=gen)
    y = torch.randint(10, (8,), device=dev, generator=gen)
    sa.train_step(x, y, F.cross_entropy)
    sb.train_step(x, y, F.cross_entropy)
    torch.cuda.synchronize()
    bad = []
    for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
        d = ((pb.grad - pa.grad).abs().max() / (pa.grad.abs().max() + 1e-12)).item()
        if d > 1e-4:
            bad.append((name, round(d, 4)))
    print(f'streams={streams} overlap={overlap} wgrad={wgrad} chunks={chunks} {checkpoint}: '
          f'{len(bad)} bad of {len(list(a.parameters()))}: {bad[:8]}', flush=True)


for cfg in [(False, False, True, 1, 'never'), (False, False, True, 4, 'never'),
            (False, False, True, 4, 'except_last'), (False, True, True, 4, 'except_last'),
            (True, False, True, 4, 'except_last'), (True, True, True, 4, 'except_last')]:
    run(*cfg)
