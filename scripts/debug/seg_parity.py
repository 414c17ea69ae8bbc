"""Per-step gradient differences of graph_cells vs eager vs an eager no-lane model (debug)."""
import copy
import sys

import torch

sys.path.insert(0, '.')
from torchgpipe_amd.parallel import PipelineStage  # noqa: E402
from tests.test_segments import _batch, _models  # noqa: E402


def errs(m1, m2):
    bad = []
    for (name, pa), pb in zip(m1.named_parameters(), m2.parameters()):
        err = ((pb.grad - pa.grad).abs().max() / (pa.grad.abs().max() + 1e-12)).item()
        if err > 1e-5:
            bad.append((name, f'{err:.2e}'))
    return bad


def run(kind, checkpoint, lanes, steps=4, opt=True):
    dev = torch.device('cuda', 0)
    base, shape, classes = _models(kind)
    a, b, c = copy.deepcopy(base), copy.deepcopy(base), copy.deepcopy(base)
    opts = dict(overlap_recompute=lanes, overlap_forward=lanes)
    sa = PipelineStage(a, [len(a)], device=dev, chunks=4, checkpoint=checkpoint, **opts)
    sb = PipelineStage(b, [len(b)], device=dev, chunks=4, checkpoint=checkpoint,
                       graph_cells=True, **opts)
    sc = PipelineStage(c, [len(c)], device=dev, chunks=4, checkpoint=checkpoint)
    os_ = [torch.optim.SGD(s.parameters(), lr=0.05) for s in (sa, sb, sc)]
    gen = torch.Generator(device=dev).manual_seed(5)
    for s in range(steps):
        x, y, loss_fn = _batch(kind, shape, classes, gen, dev)
        la = sa.train_step(x, y, loss_fn)
        lb = sb.train_step(x, y, loss_fn)
        lc = sc.train_step(x, y, loss_fn)
        torch.cuda.synchronize()
        print(kind, checkpoint, lanes, 'step', s, sb.graph_phase, 'loss', la.item(), lb.item(),
              lc.item(), '\n   lanes-eager vs graph', errs(a, b)[:5],
              '\n   plain vs lanes-eager', errs(c, a)[:5], '\n   plain vs graph', errs(c, b)[:5],
              flush=True)
        if opt:
            for o in os_:
                o.step()
                o.zero_grad(set_to_none=True)
        else:
            for p in list(a.parameters()) + list(b.parameters()) + list(c.parameters()):
                p.grad = None


for kind, ck, lanes in [('unet', 'except_last', True), ('unet', 'except_last', False),
                        ('amoebanet', 'always', True)]:
    try:
        run(kind, ck, lanes)
    except Exception:  # keep going
        import traceback
        traceback.print_exc()
