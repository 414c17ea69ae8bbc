"""Diagnostic: which part of the fused 3x3 Conv-BN-ReLU run differs from fp64 (GPU)."""
import torch
from torch import nn
import torch.nn.functional as F

from torchgpipe_amd.ops.conv import WinogradConv2d
from torchgpipe_amd.ops.fusion import bn_act


def rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm()).item()


for (n, c, hw) in [(4, 64, 28), (4, 256, 14), (4, 256, 16), (8, 256, 14)]:
    torch.manual_seed(0)
    conv = WinogradConv2d(c, c, 3, padding=1, bias=False).cuda()
    x = torch.randn(n, c, hw, hw, device='cuda', requires_grad=True)
    x64 = x.detach().double().requires_grad_(True)
    w64 = conv.weight.detach().double().requires_grad_(True)
    y = conv(x)
    y64 = F.conv2d(x64, w64, padding=1)
    g = torch.randn_like(y)
    y.backward(g)
    y64.backward(g.double())
    print(f'conv {n}x{c}x{hw}: y {rel(y, y64):.2e} dx {rel(x.grad, x64.grad):.2e} '
          f'dw {rel(conv.weight.grad, w64.grad):.2e}')
    for relu in (False, True):
        bn = nn.BatchNorm2d(c).cuda()
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.5, 0.5)
        ref = nn.BatchNorm2d(c).cuda().double()
        ref.load_state_dict(bn.state_dict())
        z = torch.randn(n, c, hw, hw, device='cuda', requires_grad=True)
        z64 = z.detach().double().requires_grad_(True)
        o = bn_act(z, bn, relu)
        o64 = ref(z64)
        if relu:
            o64 = F.relu(o64)
        g = torch.randn_like(o)
        o.backward(g)
        o64.backward(g.double())
        print(f'  bn_act relu={relu}: y {rel(o, o64):.2e} dz {rel(z.grad, z64.grad):.2e} '
              f'dgamma {rel(bn.weight.grad, ref.weight.grad):.2e}')

# the composite vs the plain fp32 layers (conditioning of x.grad)
import copy  # noqa: E402
from torchgpipe_amd.ops.fusion import BatchNormAct2d, ConvBN2d, ReLU, relink  # noqa: E402
for (n, c, hw) in [(4, 64, 28), (4, 256, 14)]:
    torch.manual_seed(0)
    seq = nn.Sequential(ConvBN2d(c, c, 3, padding=1, bias=False), BatchNormAct2d(c), ReLU()).cuda()
    with torch.no_grad():
        seq[1].weight.uniform_(0.5, 1.5)
        seq[1].bias.uniform_(-0.5, 0.5)
    relink(seq)
    ref = nn.Sequential(nn.Conv2d(c, c, 3, padding=1, bias=False), nn.BatchNorm2d(c),
                        nn.ReLU()).cuda().double()
    ref.load_state_dict(seq.state_dict())
    plain = copy.deepcopy(ref).float()
    x = torch.randn(n, c, hw, hw, device='cuda', requires_grad=True)
    x64 = x.detach().double().requires_grad_(True)
    x32 = x.detach().clone().requires_grad_(True)
    g = torch.randn(n, c, hw, hw, device='cuda')
    seq(x).backward(g)
    ref(x64).backward(g.double())
    plain(x32).backward(g)
    print(f'composite {n}x{c}x{hw}: fused dx {rel(x.grad, x64.grad):.2e}, '
          f'plain fp32 dx {rel(x32.grad, x64.grad):.2e}')
