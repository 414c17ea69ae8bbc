"""Diagnostic 2: which stage of the fused 3x3 Conv-BN-ReLU backward loses x.grad accuracy
(256 channels @ 14^2), and which parameters of the fused ResNet-50 get no gradient."""
import copy

import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd.ops.fusion import BatchNormAct2d, ConvBN2d, ReLU, bn_act, relink


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


torch.manual_seed(0)
n, c, hw = 4, 256, 14
seq = nn.Sequential(ConvBN2d(c, c, 3, padding=1, bias=False), BatchNormAct2d(c), ReLU()).cuda()
with torch.no_grad():
    seq[1].weight.uniform_(0.5, 1.5)
    seq[1].bias.uniform_(-0.5, 0.5)
relink(seq)
ref = nn.Sequential(nn.Conv2d(c, c, 3, padding=1, bias=False), nn.BatchNorm2d(c),
                    nn.ReLU()).cuda().double()
ref.load_state_dict(seq.state_dict())
x = torch.randn(n, c, hw, hw, device='cuda')
g = torch.randn(n, c, hw, hw, device='cuda')
# fp64 chain with the intermediate gradient
x64 = x.double().requires_grad_(True)
z64 = F.conv2d(x64, ref[0].weight, padding=1)
z64.retain_grad()
F.relu(ref[1](z64)).backward(g.double())
# fused chain, z's gradient captured
xf = x.clone().requires_grad_(True)
zf = seq[0].__class__.__mro__[1].forward(seq[0], xf)  # WinogradConv2d.forward: the conv only
zf.retain_grad()
bn = copy.deepcopy(seq[1])
bn_act(zf, bn, True).backward(g)
print(f'z    fused vs fp64 {rel(zf, z64):.2e}')
print(f'dz   fused BN vs fp64 {rel(zf.grad, z64.grad):.2e}')
print(f'dx   fused chain vs fp64 {rel(xf.grad, x64.grad):.2e}')
# fp32 conv backward-data (MIOpen) applied to the fused dz, and Winograd applied to fp64 dz
dx_miopen = torch.nn.grad.conv2d_input(x.shape, seq[0].weight, zf.grad, padding=1)
print(f'dx   MIOpen conv^T(fused dz) vs fp64 {rel(dx_miopen, x64.grad):.2e}')
dz64_32 = z64.grad.float()
xw = x.clone().requires_grad_(True)
zw = seq[0].__class__.__mro__[1].forward(seq[0], xw)
zw.backward(dz64_32)
print(f'dx   Winograd conv^T(fp64 dz) vs fp64 {rel(xw.grad, x64.grad):.2e}')
wdz = (ref[0].weight.norm() * z64.grad.norm()).item()
print(f'|dx| {x64.grad.norm().item():.3e}  |W||dz| ~ {wdz:.3e}')

from torchgpipe_amd.models.resnet import build_resnet  # noqa: E402
torch.manual_seed(0)
fused = build_resnet([3, 4, 6, 3], num_classes=10, fused=True).cuda()
xx = torch.randn(16, 3, 96, 96, device='cuda')
nn.functional.cross_entropy(fused(xx), torch.randint(10, (16,), device='cuda')).backward()
print('fused params without grad:', [nme for nme, p in fused.named_parameters() if p.grad is None])
