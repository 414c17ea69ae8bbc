"""ResNet-101 as a flat, skippable ``nn.Sequential`` (benchmark model).

Same structure as the reference benchmark model
(``benchmarks/models/resnet/__init__.py:18-92``, ``bottleneck.py:31-79``):
each bottleneck becomes a run of flat layers, with the residual carried by a
``@skippable`` ``Identity`` (stash) / ``Residual`` (pop) pair isolated in a
per-block namespace.  ResNet-101 = 370 layers, 44.55 M parameters.

``fused=True`` (default) keeps every layer, name and parameter but builds the convolution /
BatchNorm / ReLU layers from :mod:`torchgpipe_amd.ops.fusion`: inside one partition each
``conv, bn[, relu]`` run executes as one native op (implicit-GEMM MFMA convolution with the
BatchNorm statistics in its epilogue, or Winograd F(4x4) for the 3x3 stride-1
convolutions, then one normalise + ReLU pass), the BatchNorm and ReLU layers passing the
result through.  ``fused=False`` is the plain ``nn`` model (the numerics oracle).
"""
from collections import OrderedDict
from typing import Any, Generator, List, Optional

from torch import Tensor, nn

from torchgpipe_amd.models.flatten import flatten_sequential
from torchgpipe_amd.ops.fusion import (BatchNormAct2d, ConvBN2d, Linear, ReLU, add_relu,
                                       pending_join, relink, relu_follows)
from torchgpipe_amd.skip import Namespace, pop, skippable, stash

__all__ = ['resnet50', 'resnet101', 'build_resnet']


@skippable(stash=['identity'])
class Identity(nn.Module):
    def forward(self, x: Tensor) -> Generator:  # type: ignore[override]
        yield stash('identity', x)
        return x


@skippable(pop=['identity'])
class Residual(nn.Module):
    # with a linked ReLU after it (ops/fusion.py relink): relu(x + identity) in one pass; with
    # conv3 / bn3 linked before it too, relu(bn3(conv3(x)) + identity) as one op
    fuses_relu = True
    fuses_residual_bn = True

    def __init__(self, downsample: Optional[nn.Module] = None) -> None:
        super().__init__()
        self.downsample = downsample

    def forward(self, x: Tensor) -> Generator:  # type: ignore[override]
        identity = yield pop('identity')
        if self.downsample is not None:
            identity = self.downsample(identity)
        if relu_follows(self):
            y = pending_join(x, self, identity)
            return y if y is not None else add_relu(x, identity)
        return x + identity


def _layers(fused: bool):  # type: ignore[no-untyped-def]
    if fused:
        return ConvBN2d, BatchNormAct2d, ReLU
    return nn.Conv2d, nn.BatchNorm2d, nn.ReLU


def bottleneck(inplanes: int, planes: int, stride: int = 1,
               downsample: Optional[nn.Module] = None, inplace: bool = False,
               fused: bool = False) -> nn.Sequential:
    conv, bn, relu = _layers(fused)
    ns = Namespace()
    layers: 'OrderedDict[str, nn.Module]' = OrderedDict()
    layers['identity'] = Identity().isolate(ns)
    layers['conv1'] = conv(inplanes, planes, 1, bias=False)
    layers['bn1'] = bn(planes)
    layers['relu1'] = relu(inplace=inplace)
    layers['conv2'] = conv(planes, planes, 3, stride=stride, padding=1, bias=False)
    layers['bn2'] = bn(planes)
    layers['relu2'] = relu(inplace=inplace)
    layers['conv3'] = conv(planes, planes * 4, 1, bias=False)
    layers['bn3'] = bn(planes * 4)
    layers['residual'] = Residual(downsample).isolate(ns)
    layers['relu3'] = relu(inplace=inplace)
    return nn.Sequential(layers)


def build_resnet(layers: List[int], num_classes: int = 1000, inplace: bool = False,
                 fused: bool = True) -> nn.Sequential:
    conv, bn, relu = _layers(fused)
    inplanes = 64

    def make_layer(planes: int, blocks: int, stride: int = 1) -> nn.Sequential:
        nonlocal inplanes
        downsample = None
        if stride != 1 or inplanes != planes * 4:
            downsample = nn.Sequential(conv(inplanes, planes * 4, 1, stride=stride, bias=False),
                                       bn(planes * 4))
        seq = [bottleneck(inplanes, planes, stride, downsample, inplace, fused)]
        inplanes = planes * 4
        seq += [bottleneck(inplanes, planes, inplace=inplace, fused=fused)
                for _ in range(1, blocks)]
        return nn.Sequential(*seq)

    model = nn.Sequential(OrderedDict([
        ('conv1', conv(3, 64, kernel_size=7, stride=2, padding=3, bias=False)),
        ('bn1', bn(64)),
        ('relu', relu()),
        ('maxpool', nn.MaxPool2d(kernel_size=3, stride=2, padding=1)),
        ('layer1', make_layer(64, layers[0])),
        ('layer2', make_layer(128, layers[1], stride=2)),
        ('layer3', make_layer(256, layers[2], stride=2)),
        ('layer4', make_layer(512, layers[3], stride=2)),
        ('avgpool', nn.AdaptiveAvgPool2d((1, 1))),
        ('flat', nn.Flatten()),
        ('fc', (Linear if fused else nn.Linear)(512 * 4, num_classes)),
    ]))
    model = flatten_sequential(model)

    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)
    if fused:
        relink(model)
    return model


def resnet101(**kwargs: Any) -> nn.Sequential:
    return build_resnet([3, 4, 23, 3], **kwargs)


def resnet50(**kwargs: Any) -> nn.Sequential:
    """ResNet-50 (the reference's distributed accuracy benchmark also offers it)."""
    return build_resnet([3, 4, 6, 3], **kwargs)
