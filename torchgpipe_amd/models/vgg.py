"""VGG-16 as a flat ``nn.Sequential`` (distributed accuracy benchmark model).

Same layer sequence as the reference's distributed accuracy benchmark
(``benchmarks/distributed/accuracy/vgg/__init__.py:19-62``): thirteen 3x3 convolutions
with ReLUs and five 2x2 max-pools, one ``AdaptiveAvgPool2d(7) + Flatten`` layer, and the
4096-4096-classes classifier with two dropouts -- 39 layers, so the reference's balance
lists apply unchanged.  The dropouts are the package's Philox dropout, replayed
bit-exactly under checkpoint recomputation without touching the global RNG.
"""
from typing import List, Union

from torch import nn

from torchgpipe_amd.ops.dropout import Dropout

__all__ = ['vgg16', 'VGG16_CONFIG']

# output channels per 3x3 convolution; 'M' = 2x2 max-pool
VGG16_CONFIG: List[Union[int, str]] = [64, 64, 'M', 128, 128, 'M', 256, 256, 256, 'M',
                                       512, 512, 512, 'M', 512, 512, 512, 'M']


def vgg16(num_classes: int = 1000, inplace: bool = False, batch_norm: bool = False,
          dropout: float = 0.5) -> nn.Sequential:
    """VGG-16 (configuration D); ``batch_norm`` adds a BatchNorm2d after each convolution."""
    layers: List[nn.Module] = []
    channels = 3
    for v in VGG16_CONFIG:
        if v == 'M':
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
            continue
        assert isinstance(v, int)
        layers.append(nn.Conv2d(channels, v, kernel_size=3, padding=1))
        if batch_norm:
            layers.append(nn.BatchNorm2d(v))
        layers.append(nn.ReLU(inplace=inplace))
        channels = v
    layers.append(nn.Sequential(nn.AdaptiveAvgPool2d((7, 7)), nn.Flatten()))
    width = 4096
    layers += [nn.Linear(channels * 7 * 7, width), nn.ReLU(inplace=inplace), Dropout(dropout),
               nn.Linear(width, width), nn.ReLU(inplace=inplace), Dropout(dropout),
               nn.Linear(width, num_classes)]
    model = nn.Sequential(*layers)
    for m in model.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            nn.init.zeros_(m.bias)
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.ones_(m.weight)
            nn.init.zeros_(m.bias)
        elif isinstance(m, nn.Linear):
            nn.init.normal_(m.weight, 0.0, 0.01)
            nn.init.zeros_(m.bias)
    return model
