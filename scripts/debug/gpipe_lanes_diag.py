"""GPipe(overlap_forward=True) on one GPU: which partition's lanes change the gradients."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from torchgpipe_amd import GPipe  # noqa: E402
from torchgpipe_amd.models import unet  # noqa: E402


def run(bal_kind, lanes_on):
    torch.manual_seed(0)
    model = unet(depth=3, num_convs=2, base_channels=8)
    n = len(model)
    bal = [n] if bal_kind == 1 else [n // 2, n - n // 2]
    g = GPipe(model, bal, devices=[0] * len(bal), chunks=4, checkpoint='except_last',
              overlap_forward=bool(lanes_on))
    if lanes_on and lanes_on != 'all':
        lanes = g._forward_lanes()
        for j in range(len(bal)):
            if j not in lanes_on:
                lanes[j] = None
    gen = torch.Generator(device='cuda').manual_seed(7)
    torch.manual_seed(123)
    torch.cuda.manual_seed(123)
    x = torch.rand(8, 3, 32, 32, device='cuda', generator=gen)
    out = g(x)
    loss = F.binary_cross_entropy_with_logits(out, torch.ones_like(out))
    loss.backward()
    torch.cuda.synchronize()
    return loss.item(), {name: p.grad.clone() for name, p in g.named_parameters()}


for bal in (1, 2):
    base_l, base = run(bal, False)
    again_l, again = run(bal, False)
    print(f'bal {bal}: one-stream repeat max diff',
          max((again[k] - base[k]).abs().max().item() for k in base))
    for mode in (['all'] if bal == 1 else ['all', (0,), (1,)]):
        l, gr = run(bal, mode)
        worst = sorted(((gr[k] - base[k]).abs().max().item(), k) for k in base)[-3:]
        print(f'bal {bal} lanes {mode}: loss {l - base_l:+.2e} worst {worst}')
