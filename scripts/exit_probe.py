"""Bisect an abort at interpreter exit ('terminate called without an active exception')."""
import sys
import torch
from torch import nn
sys.path.insert(0, '.')
from torchgpipe_amd import GPipe
from torchgpipe_amd.models import unet

case = sys.argv[1]
if 'unet' in case:
    m = unet(depth=2, num_convs=1, base_channels=4)
    x = torch.rand(8, 3, 32, 32, device='cuda')
else:
    m = nn.Sequential(nn.Linear(8, 8), nn.ReLU(), nn.Linear(8, 8))
    x = torch.rand(8, 8, device='cuda')
n = len(m)
devs = [0, 0] if 'two' in case else [0]
bal = [n // 2, n - n // 2] if 'two' in case else [n]
chunks = 8 if 'many' in case else 2
g = GPipe(m, bal, devices=devs, chunks=chunks)
opt = torch.optim.SGD(g.parameters(), lr=0.1)
for _ in range(2):
    y = g(x)
    if 'bwd' in case:
        y.float().mean().backward()
        opt.step()
        opt.zero_grad()
torch.cuda.synchronize()
if 'close' in case:
    g._workers.close()
print('done', case, flush=True)
