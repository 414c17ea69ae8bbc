"""Per-step gradient differences of graph_cells vs eager (debug)."""
import copy
import sys

import torch

sys.path.insert(0, '.')
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402
from tests.test_segments import _batch, _models  # noqa: E402


def run(kind, checkpoint, lanes, steps=4):
    dev = torch.device('cuda', 0)
    base, shape, classes = _models(kind)
    a, b = copy.deepcopy(base), copy.deepcopy(base)
    opts = dict(overlap_recompute=lanes, overlap_forward=lanes)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint, **opts)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       graph_cells=True, **opts)
    gen = torch.Generator(device=dev).manual_seed(5)
    for s in range(steps):
        x, y, loss_fn = _batch(kind, shape, classes, gen, dev)
        la = sa.train_step(x, y, loss_fn)
        lb = sb.train_step(x, y, loss_fn)
        torch.cuda.synchronize()
        bad = []
        for (name, pa), pb in zip(a.named_parameters(), b.parameters()):
            err = ((pb.grad - pa.grad).abs().max() / (pa.grad.abs().max() + 1e-12)).item()
            if err > 1e-4:
                bad.append((name, round(err, 4), round(pa.grad.abs().max().item(), 6),
                            round(pb.grad.abs().max().item(), 6)))
        print(kind, checkpoint, lanes, 'step', s, sb.graph_phase, 'loss', la.item(), lb.item(),
              'bad', len(bad), bad[:6], flush=True)
        for p in list(a.parameters()) + list(b.parameters()):
            p.grad = None


for kind, ck, lanes in [('unet', 'except_last', False), ('unet', 'always', False),
                        ('unet', 'except_last', True), ('amoebanet', 'except_last', False)]:
    try:
        run(kind, ck, lanes)
    except Exception as exc:  # keep going
        import traceback
        traceback.print_exc()
