"""Layer fusion links of the ResNet model (ops/fusion.py) on the CPU: the fused layers fall
back to their plain forward and compute the plain model's function."""
import torch
from torch import nn

from torchgpipe_amd.models.resnet import build_resnet
from torchgpipe_amd.ops.fusion import BatchNormAct2d, ConvBN2d, ReLU, relink


def test_links_stay_inside_a_partition():
    model = build_resnet([1, 1, 1, 1], num_classes=10)
    layers = list(model.children())
    # conv1, bn1, relu, maxpool, then the first bottleneck
    assert relink(model) == 1 + 4 * 3 + 4  # stem + 3 per block + 4 downsamples
    first = nn.Sequential(*layers[:6])      # ... identity, conv1 of block 1 (its bn1 not)
    assert relink(first) == 1                # only the stem keeps its link
    assert '_tgpipe_link' not in layers[5].__dict__
    assert '_tgpipe_link' in layers[0].__dict__


def test_fused_model_equals_plain_model_on_cpu():
    torch.manual_seed(0)
    fused = build_resnet([1, 1, 1, 1], num_classes=10, fused=True)
    plain = build_resnet([1, 1, 1, 1], num_classes=10, fused=False)
    assert list(fused.state_dict()) == list(plain.state_dict())
    plain.load_state_dict(fused.state_dict())
    x = torch.randn(2, 3, 64, 64)
    torch.testing.assert_close(fused(x), plain(x))
    fused.eval()
    plain.eval()
    torch.testing.assert_close(fused(x), plain(x))


def test_fused_layers_are_nn_subclasses():
    assert issubclass(ConvBN2d, nn.Conv2d)
    assert issubclass(BatchNormAct2d, nn.BatchNorm2d)
    assert issubclass(ReLU, nn.ReLU)
