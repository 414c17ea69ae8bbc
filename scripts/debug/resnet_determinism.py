"""Is the fused ResNet's training step deterministic on tiny planes?  Runs the same
forward + backward twice (no pipeline) at 64x64 inputs (layer4 at 2x2) and reports, in
backward order, the first layers whose output gradient or output differs between runs."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from torchgpipe_amd.models.resnet import build_resnet  # noqa: E402


def run(model, x, y):
    outs, gouts = {}, {}
    hooks = []
    for name, m in model.named_children():
        def fwd(mod, inp, out, name=name):
            if isinstance(out, torch.Tensor):
                outs[name] = out.detach().clone()
                if out.requires_grad:
                    out.register_hook(lambda g, name=name: gouts.__setitem__(name, g.clone()))
        hooks.append(m.register_forward_hook(fwd))
    for p in model.parameters():
        p.grad = None
    loss = F.cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    for h in hooks:
        h.remove()
    return outs, gouts, {n: p.grad.clone() for n, p in model.named_parameters()}


dev = torch.device('cuda', 0)
if len(sys.argv) > 1 and sys.argv[1] == 'deterministic':
    torch.backends.cudnn.deterministic = True
    torch.backends.cudnn.benchmark = False
torch.manual_seed(0)
model = build_resnet([1, 1, 1, 1], num_classes=10).to(dev)
for size, batch in ((64, 4), (224, 4)):
    gen = torch.Generator(device=dev).manual_seed(6)
    for trial in range(4):
        x = torch.rand(batch, 3, size, size, device=dev, generator=gen)
        y = torch.randint(10, (batch,), device=dev, generator=gen)
        a = run(model, x, y)
        b = run(model, x, y)
        names = list(a[0])
        fdiff = [(n, (a[0][n] - b[0][n]).abs().max().item()) for n in names]
        first_f = next(((n, d) for n, d in fdiff if d > 0), None)
        gd = [(n, (a[1][n] - b[1][n]).abs().max().item() / (a[1][n].abs().max().item() + 1e-30))
              for n in reversed(names) if n in a[1] and n in b[1]]
        first_g = next(((n, f'{d:.1e}') for n, d in gd if d > 1e-6), None)
        worst = max(((a[2][n] - b[2][n]).abs().max().item()
                     / (a[2][n].abs().max().item() + 1e-30), n) for n in a[2])
        print(f'{size}px batch {batch} trial {trial}: first fwd diff {first_f} '
              f'first grad diff (bwd order) {first_g} worst param {worst[0]:.1e} {worst[1]}',
              flush=True)
