"""Simplified U-Net as a flat, skippable ``nn.Sequential`` (benchmark model).

Same architecture, layer order and layer names as the reference benchmark
model (``benchmarks/models/unet/__init__.py:18-148``): ``depth`` encoder
levels of ``num_convs`` × (Conv3x3 → Dropout2d(0.1) → InstanceNorm2d →
LeakyReLU(0.01)) with a ``Stash`` long skip and a 2×2 max-pool, a bottleneck
level, ``depth`` decoder levels (nearest ×2 upsample, ``PopCat`` of the skip,
convs) and a 1×1 segmentation conv.  U-Net(5, 64) = 241 layers, 232.7 M
parameters, so the reference balance tables (e.g. p8 =
``[16, 27, 31, 44, 22, 57, 27, 17]``) apply unchanged.

``fused=True`` (default) keeps the 241-layer structure but makes the
``dropout`` layer a :class:`~torchgpipe_amd.ops.fused.DropNormAct` HIP kernel
(Dropout2d + InstanceNorm2d + LeakyReLU in one pass), the ``norm`` /
``relu`` layers identities, the 3×3 convolutions
:class:`~torchgpipe_amd.ops.conv.WinogradConv2d` (Winograd F(4,3)/F(2,3) on the f32
matrix cores; same parameters as ``nn.Conv2d``), and the 3-channel input and 1×1
output convolutions the implicit-GEMM kernel (``ops.convbn.GemmConv2d``), so no
MIOpen kernel is compiled on the first step.  Because every layer stays in place, any balance
that splits a cell between partitions still computes the same function, and
the state-dict is identical (those layers have no parameters).
"""
from collections import OrderedDict
from typing import Dict, Generator, List

import torch
from torch import Tensor, nn
import torch.nn.functional as F

from torchgpipe_amd.models.flatten import flatten_sequential
from torchgpipe_amd.ops.conv import WinogradConv2d
from torchgpipe_amd.ops.convbn import GemmConv2d
from torchgpipe_amd.ops.dropout import Dropout2d
from torchgpipe_amd.ops.fused import DropNormAct
from torchgpipe_amd.ops.unet_ops import MaxPool2x2, up2x_cat
from torchgpipe_amd.skip import Namespace, pop, skippable, stash

__all__ = ['unet', 'Stash', 'PopCat', 'PopUpCat']


@skippable(stash=['skip'])
class Stash(nn.Module):
    def forward(self, input: Tensor) -> Generator:  # type: ignore[override]
        yield stash('skip', input)
        return input


@skippable(pop=['skip'])
class PopCat(nn.Module):
    def forward(self, input: Tensor) -> Generator:  # type: ignore[override]
        skipped = yield pop('skip')
        if input.shape[2:] != skipped.shape[2:]:
            pad: List[int] = []
            for have, want in reversed(list(zip(input.shape[2:], skipped.shape[2:]))):
                pad += [0, want - have]
            input = F.pad(input, pad)
        return torch.cat((input, skipped), dim=1)


@skippable(pop=['skip'])
class PopUpCat(nn.Module):
    """The decoder's ``up`` and ``skip`` layers in one pass (the preceding ``up`` layer is an
    identity): ``cat(upsample_2x(input), skipped)`` on one HIP kernel (ops/unet_ops.py)."""

    def forward(self, input: Tensor) -> Generator:  # type: ignore[override]
        skipped = yield pop('skip')
        return up2x_cat(input, skipped)


def conv_block(in_channels: int, out_channels: int, fused: bool) -> nn.Sequential:
    layers: 'OrderedDict[str, nn.Module]' = OrderedDict()
    conv = WinogradConv2d if fused else nn.Conv2d
    layers['conv'] = conv(in_channels, out_channels, kernel_size=3, padding=1, bias=False)
    if fused:
        layers['dropout'] = DropNormAct(p=0.1, eps=1e-5, negative_slope=1e-2)
        layers['norm'] = nn.Identity()
        layers['relu'] = nn.Identity()
    else:
        layers['dropout'] = Dropout2d(p=0.1)  # Philox, replayed from the checkpoint tape
        layers['norm'] = nn.InstanceNorm2d(out_channels)
        layers['relu'] = nn.LeakyReLU(negative_slope=1e-2)
    return nn.Sequential(layers)


def stacked_convs(cin: int, cmid: int, cout: int, num_convs: int, fused: bool) -> nn.Sequential:
    if num_convs == 1:
        return nn.Sequential(conv_block(cin, cout, fused))
    blocks = [conv_block(cin, cmid, fused)]
    blocks += [conv_block(cmid, cmid, fused) for _ in range(num_convs - 2)]
    blocks.append(conv_block(cmid, cout, fused))
    return nn.Sequential(*blocks)


def unet(depth: int = 5, num_convs: int = 5, base_channels: int = 64, input_channels: int = 3,
         output_channels: int = 1, fused: bool = True) -> nn.Sequential:
    """Build U-Net(depth, base_channels) as a flat skippable ``nn.Sequential``."""
    b = base_channels

    def enc(i: int) -> Dict[str, int]:
        return {'in': input_channels if i == 0 else b * 2 ** (i - 1), 'mid': b * 2 ** i,
                'out': b * 2 ** i}

    def dec(i: int) -> Dict[str, int]:
        return {'in': b * 2 ** (i + 1), 'mid': int(b * 2 ** (i - 1)),
                'out': int(b * 2 ** (i - 1))}

    neck = {'in': b * 2 ** (depth - 1), 'mid': b * 2 ** depth, 'out': b * 2 ** (depth - 1)}

    def cell(ch: Dict[str, int]) -> nn.Sequential:
        return stacked_convs(ch['in'], ch['mid'], ch['out'], num_convs, fused)

    namespaces = [Namespace() for _ in range(depth)]

    encoder = nn.Sequential(*[
        nn.Sequential(OrderedDict([
            ('encode', cell(enc(i))),
            ('skip', Stash().isolate(namespaces[i])),
            ('down', MaxPool2x2() if fused else nn.MaxPool2d(2, stride=2)),
        ])) for i in range(depth)])

    bottleneck = nn.Sequential(cell(neck))

    decoder = nn.Sequential(*[
        nn.Sequential(OrderedDict([
            ('up', nn.Identity() if fused else nn.Upsample(scale_factor=2)),
            ('skip', (PopUpCat() if fused else PopCat()).isolate(namespaces[i])),
            ('decode', cell(dec(i))),
        ])) for i in reversed(range(depth))])

    segment = (GemmConv2d if fused else nn.Conv2d)(dec(0)['out'], output_channels,
                                                   kernel_size=1, bias=False)

    model = nn.Sequential(OrderedDict([
        ('encoder', encoder),
        ('bottleneck', bottleneck),
        ('decoder', decoder),
        ('segment', segment),
    ]))
    return flatten_sequential(model)
